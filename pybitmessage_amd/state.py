"""Global run-time flags, mirroring the reference's ``src/state.py:17-21``.

``shutdown`` is set to 1 by the application's clean-shutdown path
(``src/shutdown.py:23``); every PoW loop polls it between bounded device calls and raises
``StopIteration("Interrupted")``, the contract of ``_doSafePoW``
(``src/proofofwork.py:104-109``).  Inside PyBitmessage the real ``state`` module can be
plugged in instead: ``pybitmessage_amd.proofofwork.state = <module with .shutdown>``.
"""

shutdown = 0
