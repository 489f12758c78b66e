"""The batch driver (qkd_ldpc_amd/bin/qkd_ldpc_sim, compat/qkd_ldpc_sim.cpp):
the reference's config.json -> results CSV program (src/main.cpp, config.cpp,
simulation.cpp:4-70, 140-316).

CPU: configuration validation with the reference's messages, the matrix
directory handling and the per-matrix QBER grids (--dry-run, no device).
GPU: whole runs whose CSV rows equal the oracle's batch statistics printed the
way the reference's write_file prints them, invariant under splitting the
trials over devices.
"""
import json
import math
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, write_alist

SIM = os.path.join(ROOT, "qkd_ldpc_amd", "bin", "qkd_ldpc_sim")
ALIST_NAME = "(N=10240,M=5231,R=0.49,CW=3,SEED=666).txt"

BASE_CFG = {
    "threads_number": 16,
    "trials_number": 300,
    "use_config_simulation_seed": True,
    "simulation_seed": 777,
    "interactive_mode": False,
    "sum_product_max_iterations": 50,
    "use_dense_matrices": False,
    "trace_qkd_ldpc": False,
    "trace_sum_product": False,
    "trace_sum_product_llr": False,
    "enable_sum_product_msg_llr_threshold": True,
    "sum_product_msg_llr_threshold": 100.0,
    "code_rate_QBER_parameters": [
        {"code_rate": 0.36, "QBER_begin": 0.12, "QBER_end": 0.135, "QBER_step": 0.0005},
        {"code_rate": 0.58, "QBER_begin": 0.03, "QBER_end": 0.06, "QBER_step": 0.01},
        {"code_rate": 0.95, "QBER_begin": 0.005, "QBER_end": 0.05, "QBER_step": 0.0005},
    ],
}


@pytest.fixture(scope="module")
def sim_bin():
    if not os.path.exists(SIM):
        from qkd_ldpc_amd.build import build
        build()
    return SIM


def make_root(tmp_path, golden_code, cfg, dense=None):
    root = tmp_path
    (root / "alist_sparse_matrices").mkdir(exist_ok=True)
    g = golden_code
    write_alist(str(root / "alist_sparse_matrices" / ALIST_NAME), int(g["dims"][0]), int(g["dims"][1]),
                g["bit_off"], g["bit_idx"], g["chk_off"], g["chk_idx"])
    if dense is not None:
        (root / "dense_matrices").mkdir(exist_ok=True)
        for name, H in dense.items():
            with open(root / "dense_matrices" / f"{name}.txt", "w") as f:
                for row in H:
                    f.write(" ".join(str(int(x)) for x in row) + "\n")
    with open(root / "config.json", "w") as f:
        json.dump(cfg, f, indent=2)
    return root


def run(sim_bin, root, *extra):
    return subprocess.run([sim_bin, "--root", str(root), *extra], capture_output=True, text=True, timeout=600)


def ref_grid(rate, params):
    """get_rate_based_QBER_range (simulation.cpp:48-70) in Python doubles (C round:
    half away from zero)."""
    for p in sorted(params, key=lambda p: p["code_rate"]):
        if rate <= p["code_rate"]:
            x = (p["QBER_end"] - p["QBER_begin"]) / p["QBER_step"]
            steps = int(math.floor(x + 0.5))
            return [p["QBER_begin"] + j * p["QBER_step"] for j in range(steps)]
    return []


# ---- CPU ----------------------------------------------------------------------------

@pytest.mark.parametrize("patch,message", [
    ({"threads_number": 0}, "Number of threads must be >= 1!"),
    ({"trials_number": 0}, "Number of trials must be >= 1!"),
    ({"sum_product_max_iterations": 0}, "Minimum number of sum-product iterations must be >= 1!"),
    ({"sum_product_msg_llr_threshold": 0.0}, "Sum-product message LLR threshold must be > 0!"),
    ({"code_rate_QBER_parameters": []}, "Array with code rate and QBER parameters is empty!"),
    ({"code_rate_QBER_parameters": [{"code_rate": 1.0, "QBER_begin": 0.1, "QBER_end": 0.2, "QBER_step": 0.01}]},
     "Code rate(R) must be: 0 < R < 1!"),
    ({"code_rate_QBER_parameters": [{"code_rate": 0.5, "QBER_begin": 0.2, "QBER_end": 0.1, "QBER_step": 0.01}]},
     "Invalid QBER begin or end parameters"),
    ({"code_rate_QBER_parameters": [{"code_rate": 0.5, "QBER_begin": 0.1, "QBER_end": 0.2, "QBER_step": 0.0}]},
     "QBER step must be > 0!"),
    ({"code_rate_QBER_parameters": [{"code_rate": 0.5, "QBER_begin": 0.1, "QBER_end": 0.2, "QBER_step": 0.5}]},
     "QBER step is too large."),
])
def test_config_validation_messages(sim_bin, tmp_path, golden_code, patch, message):
    cfg = dict(BASE_CFG, **patch)
    root = make_root(tmp_path, golden_code, cfg)
    r = run(sim_bin, root, "--dry-run")
    assert r.returncode == 1
    assert "An error occurred while reading a configuration parameter." in r.stderr
    assert message in r.stderr


def test_config_missing_key_and_bad_json(sim_bin, tmp_path, golden_code):
    cfg = dict(BASE_CFG)
    del cfg["trace_sum_product"]
    root = make_root(tmp_path, golden_code, cfg)
    r = run(sim_bin, root, "--dry-run")
    assert r.returncode == 1 and "trace_sum_product" in r.stderr
    (root / "config.json").write_text('{"threads_number": 16, ')
    r = run(sim_bin, root, "--dry-run")
    assert r.returncode == 1 and "parse_error" in r.stderr
    os.remove(root / "config.json")
    r = run(sim_bin, root, "--dry-run")
    assert r.returncode == 1 and "Configuration file not found" in r.stderr


def test_threshold_off_skips_its_value(sim_bin, tmp_path, golden_code):
    """config.cpp reads sum_product_msg_llr_threshold only when it is enabled."""
    cfg = dict(BASE_CFG, enable_sum_product_msg_llr_threshold=False)
    del cfg["sum_product_msg_llr_threshold"]
    r = run(sim_bin, make_root(tmp_path, golden_code, cfg), "--dry-run")
    assert r.returncode == 0, r.stderr


def test_matrix_directory_errors(sim_bin, tmp_path, golden_code):
    root = make_root(tmp_path, golden_code, BASE_CFG)
    os.remove(root / "alist_sparse_matrices" / ALIST_NAME)
    r = run(sim_bin, root, "--dry-run")
    assert r.returncode == 1 and "Matrix folder is empty" in r.stderr
    os.rmdir(root / "alist_sparse_matrices")
    r = run(sim_bin, root, "--dry-run")
    assert r.returncode == 1 and "Directory doesn't exist." in r.stderr



def test_dry_run_grids_match_reference_rule(sim_bin, tmp_path, golden_code, dense_codes):
    """Each matrix gets the grid of the first (sorted) parameter row whose code
    rate is >= its own; for the reference's own config.json rows, bit-exact."""
    ref_rows = [  # the reference's config.json:14-28
        {"code_rate": 0.95, "QBER_begin": 0.005, "QBER_end": 0.05, "QBER_step": 0.0005},
        {"code_rate": 0.36, "QBER_begin": 0.12, "QBER_end": 0.135, "QBER_step": 0.0005},
        {"code_rate": 0.58, "QBER_begin": 0.06, "QBER_end": 0.075, "QBER_step": 0.0005},
    ]
    for dense in (False, True):
        cfg = dict(BASE_CFG, code_rate_QBER_parameters=ref_rows, use_dense_matrices=dense)
        root = make_root(tmp_path, golden_code, cfg, dense=dense_codes)
        r = run(sim_bin, root, "--dry-run")
        assert r.returncode == 0, r.stderr
        lines = r.stdout.strip().splitlines()
        assert len(lines) == (len(dense_codes) if dense else 1)
        for line in lines:
            head, grid = line.split(" QBER")
            fields = dict(kv.split("=") for kv in head.split()[1:])
            n, m = int(fields["N"]), int(fields["M"])
            rate = 1.0 - m / n
            assert float(fields["R"]) == rate
            got = [float(x) for x in grid.split()]
            assert got == ref_grid(rate, ref_rows), line
        if not dense:
            assert len(got) == 30 and got[0] == 0.06


def test_no_device_is_an_error(sim_bin, tmp_path, golden_code):
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is visible")
    except Exception:
        pass
    r = run(sim_bin, make_root(tmp_path, golden_code, BASE_CFG))
    assert r.returncode == 1 and "HIP device" in r.stderr


# ---- GPU ----------------------------------------------------------------------------

def fmt(x):
    """std::ostream's default formatting of a double (%g, 6 significant digits)."""
    return f"{x:g}"


@pytest.mark.gpu
def test_batch_run_csv_equals_oracle(sim_bin, tmp_path, golden_code, oracle_mod, oracle_code):
    cfg = dict(BASE_CFG)
    root = make_root(tmp_path, golden_code, cfg)
    r = run(sim_bin, root, "--quiet")
    assert r.returncode == 0, r.stderr
    name = "ldpc(trial_num=300,max_sum_prod_iters=50,seed=777).csv"
    path = root / "results" / name
    text = path.read_text(encoding="utf-8")
    lines = text.splitlines()
    assert lines[0] == ("№;MATRIX_FILENAME;TYPE;CODE_RATE;M;N;QBER;ITERATIONS_SUCCESSFUL_SP_MEAN;"
                        "ITERATIONS_SUCCESSFUL_SP_STD_DEV;ITERATIONS_SUCCESSFUL_SP_MIN;"
                        "ITERATIONS_SUCCESSFUL_SP_MAX;RATIO_TRIALS_SUCCESSFUL_SP;RATIO_TRIALS_SUCCESSFUL_LDPC;FER")
    n, m = 10240, 5231
    rate = 1.0 - m / n
    grid = ref_grid(rate, cfg["code_rate_QBER_parameters"])
    assert len(grid) == 3 and len(lines) == 1 + len(grid)
    seeds = oracle_mod.seeds(777, cfg["trials_number"])
    for s, q in enumerate(grid):
        t = oracle_code.trials(q, seeds, s, 50, 100.0, True)
        st = oracle_mod.batch_stats(t["iters"], t["sp_ok"], t["key_ok"], t["exact_q"], 300, 50)
        want = ";".join([str(s), ALIST_NAME, "irregular", fmt(rate), str(m), str(n), fmt(st["initial_QBER"]),
                         fmt(st["iterations_successful_sp_mean"]), fmt(st["iterations_successful_sp_std_dev"]),
                         str(st["iterations_successful_sp_min"]), str(st["iterations_successful_sp_max"]),
                         fmt(st["ratio_trials_successful_sp"]), fmt(st["ratio_trials_successful_ldpc"]),
                         fmt(1.0 - st["ratio_trials_successful_ldpc"])])
        assert lines[1 + s] == want
    # a second run keeps the first file and writes "_1" (write_file's numbering)
    r2 = run(sim_bin, root, "--quiet", "--devices", "0,0,0")
    assert r2.returncode == 0, r2.stderr
    second = root / "results" / name.replace(").csv", ")_1.csv")
    assert second.read_text(encoding="utf-8") == text      # split over three shards: same rows


# ---- interactive mode (simulation.cpp:73-137) ------------------------------------------

INTERACTIVE_CFG = dict(BASE_CFG, interactive_mode=True, code_rate_QBER_parameters=[
    {"code_rate": 0.58, "QBER_begin": 0.06, "QBER_end": 0.0745, "QBER_step": 0.0005}])   # config.json:20-23


def interactive_lines(res, n_points):
    """The lines QKD_LDPC_interactive_simulation prints per point (:100-132)."""
    out = []
    for i in range(n_points):
        out += [f"№:{i + 1}", f"Actual QBER: {float(res['exact_q'][i])!r}",
                f"Number of errors in a key: {res['errors'][i]}",
                f"Iterations performed: {res['iters'][i]}",
                "Error reconciliation SUCCESSFUL" if res["sp_ok"][i] and res["key_ok"][i]
                else "Error reconciliation FAILED"]
    return out


def test_interactive_rejects_bad_file_number(sim_bin, tmp_path, golden_code):
    root = make_root(tmp_path, golden_code, INTERACTIVE_CFG)
    r = subprocess.run([sim_bin, "--root", str(root)], input="7\n", capture_output=True, text=True, timeout=120)
    assert r.returncode == 1 and "Wrong file number." in r.stderr
    assert "INTERACTIVE MODE" in r.stdout and f"1. {ALIST_NAME}" in r.stdout


@pytest.mark.gpu
def test_interactive_driver_matches_oracle(sim_bin, tmp_path, golden_code, oracle_code, oracle_mod):
    """The reference's default grid for the R=0.49 code (30 points, QBER 0.06-0.0745)
    with one shared key stream: every printed line equals the oracle's restatement."""
    root = make_root(tmp_path, golden_code, INTERACTIVE_CFG)
    r = subprocess.run([sim_bin, "--root", str(root)], input="1\n", capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    rate = 1 - 5231 / 10240
    grid = ref_grid(rate, INTERACTIVE_CFG["code_rate_QBER_parameters"])
    assert len(grid) == 29
    want = oracle_mod.interactive(oracle_code, 777, grid, 50, 100.0, True)
    assert want["stop"] == -1
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert lines[:3] == ["INTERACTIVE MODE", "Choose file: ", f"1. {ALIST_NAME}"]
    assert lines[3] == "Matrix H is irregular."
    assert lines[4:] == interactive_lines(want, len(grid))


@pytest.mark.gpu
def test_interactive_api_and_too_small_qber(golden_code, oracle_code, oracle_mod, dense_codes):
    """qkd_interactive_batch through Python: per-point results equal the oracle's,
    the stream continues across points (point 2 differs from a fresh seed), and a
    point with floor(N q) = 0 stops the run there with the earlier points done."""
    import qkd_ldpc_amd as Q
    g = golden_code
    H = Q.HMatrix.from_check_lists(10240, g["chk_off"], g["chk_idx"])
    qs = [0.02, 0.05, 0.08, 0.03, 0.11]
    got = Q.interactive_simulation(H, 12345, qs)
    want = oracle_mod.interactive(oracle_code, 12345, qs)
    for k in ("iterations", "errors"):
        assert got[k].tolist() == want["iters" if k == "iterations" else k].tolist(), k
    assert got["syndromes_match"].tolist() == want["sp_ok"].tolist()
    assert got["keys_match"].tolist() == want["key_ok"].tolist()
    assert got["exact_qber"].tolist() == want["exact_q"].tolist()
    # the dense N=10 code: 0.05 * 10 floors to 0 at the third point
    name = "(N=10,K=5,M=5,R=0.5).txt"
    Hd = Q.HMatrix.from_dense_array(dense_codes[name])
    od = oracle_mod.Code.from_dense(dense_codes[name])
    qd = [0.2, 0.1, 0.05, 0.3]
    want = oracle_mod.interactive(od, 777, qd, 100, 100.0, True)
    assert want["stop"] == 2
    with pytest.raises(Q.QkdError) as ei:
        Q.interactive_simulation(Hd, 777, qd, 100)
    part = ei.value.partial
    assert ei.value.status == Q._native.ERR_QBER_TOO_SMALL and part["points_done"] == 2
    assert part["iterations"].tolist() == want["iters"][:2].tolist()
    assert part["success"].tolist() == (want["sp_ok"] & want["key_ok"])[:2].tolist()
