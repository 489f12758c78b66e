"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (needs /root/reference for the matrix files):

    python tests/golden/gen_golden.py [--skip-config3]

Outputs (all data, no reference source):
  code_n10240.npz      adjacency of alist (N=10240,M=5231,R=0.49,CW=3,SEED=666)
                       as offset/index arrays, exactly as the reference reads it
                       (array_and_matrix_operations.cpp:109-292), so the GPU box
                       (which has no /root/reference) gets the benchmark code.
  dense_codes.json     the three dense textbook matrices (dense_matrices/*.txt).
  oracle_vectors.npz   per-frame oracle results (checked against the reference
                       pins in reference_probe.json before writing):
                         c2_iters/c2_sp/c2_ko/c2_q  config 2, 4096 frames
                         c3_iters/c3_sp/c3_ko/c3_q  config 3, 8 points x 10000
                         kg_*                       keygen vectors (packed bits)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

REF = "/root/reference"
ALIST = os.path.join(REF, "alist_sparse_matrices", "(N=10240,M=5231,R=0.49,CW=3,SEED=666).txt")


def read_dense(path):
    rows = [[int(x) for x in line.split()] for line in open(path) if line.strip()]
    return rows


def qber_grid(begin, end, step):
    # get_rate_based_QBER_range, simulation.cpp:55-60 (round, end exclusive)
    steps = int(round((end - begin) / step))
    return [begin + j * step for j in range(steps)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skip-config3", action="store_true")
    args = ap.parse_args()
    probe = json.load(open(os.path.join(HERE, "reference_probe.json")))

    code = O.Code.from_alist(ALIST)
    bo, bi, co, ci = code.lists()
    np.savez_compressed(os.path.join(HERE, "code_n10240.npz"), bit_off=bo, bit_idx=bi,
                        chk_off=co, chk_idx=ci,
                        dims=np.array([code.n, code.m, code.max_dv, code.max_dc], np.int32))

    dense = {}
    for name in sorted(os.listdir(os.path.join(REF, "dense_matrices"))):
        dense[name] = read_dense(os.path.join(REF, "dense_matrices", name))
    json.dump(dense, open(os.path.join(HERE, "dense_codes.json"), "w"), indent=0)

    out = {}
    seeds = O.seeds(777, 10000)
    assert int(seeds[0]) == int(probe["seeds_777_first"])

    # keygen vectors
    kg_seeds = seeds[:16]
    kg_q = [0.02, 0.08, 0.0001, 0.5]
    A, B, Q = [], [], []
    for qn in kg_q:
        for s in kg_seeds:
            a, b, q = O.keygen(int(s), code.n, qn)
            A.append(np.packbits(a.astype(np.uint8)))
            B.append(np.packbits(b.astype(np.uint8)))
            Q.append(q)
    out["kg_seeds"] = kg_seeds
    out["kg_qnom"] = np.repeat(np.array(kg_q), len(kg_seeds))
    out["kg_alice"] = np.stack(A)
    out["kg_bob"] = np.stack(B)
    out["kg_q"] = np.array(Q)

    # config 2
    t = time.time()
    r = code.trials(0.02, seeds[:4096], 0, 50, 100.0, True)
    st = O.batch_stats(r["iters"], r["sp_ok"], r["key_ok"], r["exact_q"], 4096, 50)
    p2 = probe["config2"]
    assert st["sum_iters_sp"] == p2["sum_iterations"], st
    assert round(st["iterations_successful_sp_std_dev"], 6) == p2["std_6sig"], st
    assert st["fer"] == p2["fer"]
    print(f"config2 ok ({time.time() - t:.1f}s): {st}")
    out["c2_iters"] = r["iters"].astype(np.uint8)
    out["c2_sp"] = r["sp_ok"]
    out["c2_ko"] = r["key_ok"]
    out["c2_q"] = r["exact_q"][:1]

    if not args.skip_config3:
        p3 = probe["config3"]
        grid = qber_grid(p3["qber_begin"], p3["qber_end"], p3["qber_step"])
        its, sps, kos, qs = [], [], [], []
        for s, qn in enumerate(grid):
            t = time.time()
            r = code.trials(qn, seeds[:10000], s, 50, 100.0, True)
            st = O.batch_stats(r["iters"], r["sp_ok"], r["key_ok"], r["exact_q"], 10000, 50)
            pp = p3["points"][s]
            assert round(st["initial_QBER"], 5) == round(pp["qber_actual"], 5), (st, pp)
            assert abs(st["iterations_successful_sp_mean"] - pp["mean_it"]) <= 0.0005 + 1e-9, (st, pp)
            assert abs(st["fer"] - pp["fer"]) < 1e-12, (st, pp)
            print(f"config3 point {s} q={qn} ok ({time.time() - t:.1f}s): mean "
                  f"{st['iterations_successful_sp_mean']:.4f} fer {st['fer']}")
            its.append(r["iters"].astype(np.uint8))
            sps.append(r["sp_ok"])
            kos.append(r["key_ok"])
            qs.append(r["exact_q"][0])
        out["c3_qnom"] = np.array(grid)
        out["c3_iters"] = np.stack(its)
        out["c3_sp"] = np.stack(sps)
        out["c3_ko"] = np.stack(kos)
        out["c3_q"] = np.array(qs)
    else:
        old = os.path.join(HERE, "oracle_vectors.npz")
        if os.path.exists(old):
            with np.load(old) as z:
                for k in ("c3_qnom", "c3_iters", "c3_sp", "c3_ko", "c3_q"):
                    if k in z:
                        out[k] = z[k]

    np.savez_compressed(os.path.join(HERE, "oracle_vectors.npz"), **out)
    print("wrote", os.path.join(HERE, "oracle_vectors.npz"))


if __name__ == "__main__":
    main()
