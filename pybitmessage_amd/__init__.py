"""pybitmessage_amd -- MI355X-native proof-of-work engine for PyBitmessage.

The hot path (``proofofwork.run`` / ``run_batch``) runs hand-written gfx950 HIP kernels in
``libbmpow_hip.so`` (``csrc/``, C ABI in ``include/bmpow.h``).  See DESIGN.md.
"""
__all__ = ['proofofwork', 'state', 'targets']
