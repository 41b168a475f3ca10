#!/usr/bin/env python3
"""Generate ``tests/golden/sender_targets_ref.json`` by running the REFERENCE's own sender-side
target expressions.

Run in the build container only (needs /root/reference, read-only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_target_golden.py

``class_singleWorker`` does not import under Python 3 here (its ``inventory`` -> ``storage``
chain raises ImportError), so this script takes the two expressions out of the module's source
with ``ast`` and evaluates exactly those nodes, compiled under the module's own
``from __future__ import division``:

* the ``target = 2 ** 64 / (...)`` statement of ``_doPOWDefaults``
  (src/class_singleWorker.py:222-230), evaluated with ``defaults`` bound to the reference's
  ``defaults`` module (network defaults, then the test-mode /100 of bitmessagemain.py:167-172)
  and the given ``payload`` and ``TTL`` (ints, and the float TTLs requestPubKey produces);
* the ``target = 2 ** 64 / (...)`` statement of ``sendMsg`` (:1256-1264), evaluated with the
  recipient's ``requiredAverageProofOfWorkNonceTrialsPerByte`` /
  ``requiredPayloadLengthExtraBytes``.

The fixture holds the float targets (``float.hex``) the reference hands to ``proofofwork.run``,
which ``int()``s them (src/proofofwork.py:293).
"""
import ast
import json
import os
import random
import sys

REF = '/root/reference/src'
HERE = os.path.dirname(os.path.abspath(__file__))


def target_expr(tree, func):
    for node in ast.walk(tree):
        if isinstance(node, ast.FunctionDef) and node.name == func:
            for sub in ast.walk(node):
                if isinstance(sub, ast.Assign) and len(sub.targets) == 1 and \
                        isinstance(sub.targets[0], ast.Name) and sub.targets[0].id == 'target':
                    return compile(ast.Expression(sub.value), '<%s target>' % func, 'eval',
                                   flags=__import__('__future__').division.compiler_flag, dont_inherit=True)
    raise SystemExit('no target statement in %s' % func)


def main():
    sys.path.insert(0, REF)
    import defaults  # the reference's module: networkDefault* constants (src/defaults.py)
    src = open(os.path.join(REF, 'class_singleWorker.py')).read()
    tree = ast.parse(src)
    pow_defaults = target_expr(tree, '_doPOWDefaults')
    send_msg = target_expr(tree, 'sendMsg')
    rng = random.Random(20250216)
    cases = []
    lens = [46, 54, 100, 150, 200, 512, 1000, 1024, 4096, 16384, 65536, 262144] + [rng.randrange(1, 262145)
                                                                                    for _ in range(40)]
    ttls = [300, 3600, 86400, 4 * 86400, 345600, 604800, 2419200, 28 * 86400 - 300, 28 * 86400 + 299,
            216000.0 + 17, 432000.0 - 120, 864000.0, 2419200.0 + 5] + [rng.randrange(300, 2419500) for _ in range(20)]
    saved = (defaults.networkDefaultProofOfWorkNonceTrialsPerByte, defaults.networkDefaultPayloadLengthExtraBytes)
    for mode, div in (('default', 1), ('test', 100)):
        defaults.networkDefaultProofOfWorkNonceTrialsPerByte = int(saved[0] / div)
        defaults.networkDefaultPayloadLengthExtraBytes = int(saved[1] / div)
        for L in lens:
            for ttl in rng.sample(ttls, 6):
                t = eval(pow_defaults, {'defaults': defaults}, {'payload': b'\0' * L, 'TTL': ttl})  # noqa: S307
                cases.append({'kind': 'pow_defaults', 'mode': mode, 'L': L, 'ttl': ttl,
                              'ntpb': defaults.networkDefaultProofOfWorkNonceTrialsPerByte,
                              'extra': defaults.networkDefaultPayloadLengthExtraBytes,
                              'target_float': t.hex(), 'target': int(t)})
    defaults.networkDefaultProofOfWorkNonceTrialsPerByte, defaults.networkDefaultPayloadLengthExtraBytes = saved
    for L in lens[:30]:
        for ntpb, extra in ((1000, 1000), (2000, 1500), (20000, 1000), (1001, 999999), (10, 10)):
            ttl = rng.choice([t for t in ttls if isinstance(t, int)])
            t = eval(send_msg, {}, {'encryptedPayload': b'\0' * L, 'TTL': ttl,  # noqa: S307
                                    'requiredAverageProofOfWorkNonceTrialsPerByte': ntpb,
                                    'requiredPayloadLengthExtraBytes': extra})
            cases.append({'kind': 'send_msg', 'L': L, 'ttl': ttl, 'ntpb': ntpb, 'extra': extra,
                          'target_float': t.hex(), 'target': int(t)})
    out = {'source': 'src/class_singleWorker.py _doPOWDefaults (:222-230) and sendMsg (:1256-1264) target '
                     'statements, evaluated by tests/golden/make_target_golden.py', 'cases': cases}
    with open(os.path.join(HERE, 'sender_targets_ref.json'), 'w') as f:
        json.dump(out, f, indent=0)
    print('wrote %d cases' % len(cases))


if __name__ == '__main__':
    main()
