"""Every FNV word-hash definition tried against SURVEY.md section 4 fingerprint c2b#1 of config-2
frame 0 (none matches; recorded in tests/golden/reference_probe.json). Test tooling: uses the oracle."""
import sys, itertools
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import numpy as np
from oracle import oracle as O
g = dict(np.load('tests/golden/code_n10240.npz'))
code = O.Code.from_lists(g)
bo, bi, co, ci = g['bit_off'], g['bit_idx'], g['chk_off'], g['chk_idx']
seed = int(O.seeds(777, 1)[0])
a, b, q = O.keygen(seed, 10240, 0.02)
print('errors', int((a ^ b).sum()), q)
syn = code.syndrome(a)
target = 0x00d2fe5b7758b063
M64 = (1 << 64) - 1
def fnv1a_words(ws):
    h = 0xcbf29ce484222325
    for u in ws: h = ((h ^ int(u)) * 0x100000001b3) & M64
    return h
def fnv1_words(ws):
    h = 0xcbf29ce484222325
    for u in ws: h = ((h * 0x100000001b3) & M64) ^ int(u)
    return h
def fnv1a_bytes(bs):
    h = 0xcbf29ce484222325
    for x in bs: h = ((h ^ x) * 0x100000001b3) & M64
    return h
def fnv1_bytes(bs):
    h = 0xcbf29ce484222325
    for x in bs: h = ((h * 0x100000001b3) & M64) ^ x
    return h
# check-major reorder of a bit-major c2b array
pos = {}
for i in range(10240):
    for k in range(bo[i], bo[i+1]): pos[(int(bi[k]), i)] = k
cm_idx = np.array([pos[(j, int(ci[k]))] for j in range(5231) for k in range(co[j], co[j+1])])
found = False
for qq_name, qq in [('exact', q), ('nominal', 0.02)]:
    lp = np.log((1 - qq) / qq)
    llr = np.where(b == 1, -lp, lp)
    r = code.decode(llr, syn, 50, 100.0, True, fingerprints=True, etrace=True)
    E = r['etrace'][0]
    for order_name, arr in [('bitmajor', E), ('checkmajor', E[cm_idx])]:
        ws = arr.view(np.uint64)
        cands = {
            'fnv1a_w': fnv1a_words(ws), 'fnv1_w': fnv1_words(ws),
            'fnv1a_b_le': fnv1a_bytes(arr.astype('<f8').tobytes()), 'fnv1_b_le': fnv1_bytes(arr.astype('<f8').tobytes()),
            'fnv1a_b_be': fnv1a_bytes(arr.astype('>f8').tobytes()),
            'fnv1a_val': fnv1a_words([int(x) & M64 for x in arr.astype(np.int64)]),
        }
        for k, v in cands.items():
            flag = '  <== MATCH' if v == target else ''
            print(qq_name, order_name, k, hex(v), flag)
            found |= v == target
print('found', found, 'oracle fp', hex(r['fingerprints'][0]))
