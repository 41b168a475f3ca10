#!/usr/bin/env python3
"""Generate ``tests/golden/sender_targets_ref.json`` by running the REFERENCE's own sender-side
target expressions.

Run in the build container only (needs /root/reference, read-only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_target_golden.py

Nothing of the reference is imported, compiled or evaluated: the reference tree is untrusted input.
The script reads its sources as text and walks their syntax trees --

* the ``networkDefault*`` constants are ``ast.literal_eval``-ed from their assignments in
  src/defaults.py;
* the ``target = 2 ** 64 / (...)`` statements of ``_doPOWDefaults`` (src/class_singleWorker.py:
  222-230) and ``sendMsg`` (:1256-1264) are taken out of class_singleWorker.py with ``ast`` and
  checked structurally: only numbers, names, ``defaults.<attr>``, ``len(name)`` and the binary
  operators + - * / ** may appear;
* a ten-line interpreter of exactly that node set evaluates them with the module's own
  ``from __future__ import division`` semantics (``/`` is true division), with ``defaults`` bound to
  the constants above (network defaults, then the test-mode /100 of bitmessagemain.py:167-172) and
  the given ``payload`` / ``TTL`` (ints, and the float TTLs requestPubKey produces) or the
  recipient's ``requiredAverageProofOfWorkNonceTrialsPerByte`` / ``requiredPayloadLengthExtraBytes``.

The fixture holds the float targets (``float.hex``) the reference hands to ``proofofwork.run``,
which ``int()``s them (src/proofofwork.py:293).
"""
import ast
import json
import operator
import os
import random

REF = '/root/reference/src'
HERE = os.path.dirname(os.path.abspath(__file__))

_BINOPS = {ast.Add: operator.add, ast.Sub: operator.sub, ast.Mult: operator.mul,
           ast.Div: operator.truediv,  # the module's `from __future__ import division` (:7)
           ast.Pow: operator.pow}


def target_expr(tree, func):
    """The value node of the ``target = ...`` statement in function ``func`` (not evaluated)."""
    for node in ast.walk(tree):
        if isinstance(node, ast.FunctionDef) and node.name == func:
            for sub in ast.walk(node):
                if isinstance(sub, ast.Assign) and len(sub.targets) == 1 and \
                        isinstance(sub.targets[0], ast.Name) and sub.targets[0].id == 'target':
                    check_shape(sub.value)
                    return sub.value
    raise SystemExit('no target statement in %s' % func)


def check_shape(node):
    """Only arithmetic on numbers, names, defaults.<attr> and len(<name>) -- refuse anything else."""
    for n in ast.walk(node):
        ok = isinstance(n, (ast.Expression, ast.BinOp, ast.Name, ast.Load, ast.Attribute, ast.Call)) or \
            type(n) in _BINOPS or (isinstance(n, ast.Constant) and type(n.value) in (int, float))
        if isinstance(n, ast.Attribute):
            ok = isinstance(n.value, ast.Name) and n.value.id == 'defaults'
        if isinstance(n, ast.Call):
            ok = isinstance(n.func, ast.Name) and n.func.id == 'len' and len(n.args) == 1 and not n.keywords \
                and isinstance(n.args[0], ast.Name)
        if not ok:
            raise SystemExit('unexpected node in a target expression: %s' % ast.dump(n))


def evaluate(node, env):
    """The target expression's value, by our own interpreter of check_shape's node set."""
    if isinstance(node, ast.Constant):
        return node.value
    if isinstance(node, ast.Name):
        return env[node.id]
    if isinstance(node, ast.Attribute):
        return env['defaults.' + node.attr]
    if isinstance(node, ast.Call):
        return len(env[node.args[0].id])
    return _BINOPS[type(node.op)](evaluate(node.left, env), evaluate(node.right, env))


def network_defaults():
    """networkDefault* constants of src/defaults.py, literal_eval-ed from their assignments."""
    tree = ast.parse(open(os.path.join(REF, 'defaults.py')).read())
    out = {}
    for node in tree.body:
        if isinstance(node, ast.Assign) and len(node.targets) == 1 and isinstance(node.targets[0], ast.Name):
            name = node.targets[0].id
            if name in ('networkDefaultProofOfWorkNonceTrialsPerByte', 'networkDefaultPayloadLengthExtraBytes'):
                out[name] = ast.literal_eval(node.value)
    assert len(out) == 2, out
    return out


def main():
    base = network_defaults()
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
    for mode, div in (('default', 1), ('test', 100)):
        ntpb = int(base['networkDefaultProofOfWorkNonceTrialsPerByte'] / div)
        extra = int(base['networkDefaultPayloadLengthExtraBytes'] / div)
        for L in lens:
            for ttl in rng.sample(ttls, 6):
                t = evaluate(pow_defaults, {'defaults.networkDefaultProofOfWorkNonceTrialsPerByte': ntpb,
                                            'defaults.networkDefaultPayloadLengthExtraBytes': extra,
                                            'payload': b'\0' * L, 'TTL': ttl})
                cases.append({'kind': 'pow_defaults', 'mode': mode, 'L': L, 'ttl': ttl, 'ntpb': ntpb, 'extra': extra,
                              'target_float': t.hex(), 'target': int(t)})
    for L in lens[:30]:
        for ntpb, extra in ((1000, 1000), (2000, 1500), (20000, 1000), (1001, 999999), (10, 10)):
            ttl = rng.choice([t for t in ttls if isinstance(t, int)])
            t = evaluate(send_msg, {'encryptedPayload': b'\0' * L, 'TTL': ttl,
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
