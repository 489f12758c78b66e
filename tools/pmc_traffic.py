"""HBM-side traffic of the decode kernel per launch from rocprofv3 --pmc passes
(tools/gpu_pmc.sh: pass 1 FETCH_SIZE, pass 2 WRITE_SIZE), corrected as
/opt/skills/guides/MI355X_MICROARCH.md prescribes for gfx950: FETCH_SIZE (KB)
reports 1/2 of the bytes of wide reads -> x2; WRITE_SIZE (KB) as is.

    python tools/pmc_traffic.py gpurun_out/pmc_1 gpurun_out/pmc_2 profiles/r01_pmc_decode.json [gpurun_out/pmc_3]

With the third directory (tools/gpu_pmc.sh pass 3: SQ_ACTIVE_INST_VALU,
SQ_INSTS_VALU, GRBM_GUI_ACTIVE ...) the file also records the VALU busy
fraction: SQ_ACTIVE_INST_VALU x 4 cycles / (GRBM_GUI_ACTIVE / XCDs x SIMDs).
"""
import csv
import json
import os
import sys


# the headline kernel: the speculative split-store decoder, keys path, binary64
KERNEL = os.environ.get("QKD_PMC_KERNEL", "decode_split_kernel<1, 0, 6, true, 1>")


def per_launch(d, counter):
    vals = []
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals), len(vals)


def main():
    fetch_kb, nf = per_launch(sys.argv[1], "FETCH_SIZE")
    write_kb, nw = per_launch(sys.argv[2], "WRITE_SIZE")
    out = {
        "kernel": KERNEL + " (qkd_qkd_ldpc_batch, 4096 frames, QBER 0.02)",
        "fetch_size_kb": fetch_kb,
        "write_size_kb": write_kb,
        "launches": [nf, nw],
        "correction": "FETCH_SIZE x2 (gfx950), WRITE_SIZE x1; KB = 1024 B",
        "hbm_bytes_per_launch": fetch_kb * 1024 * 2 + write_kb * 1024,
    }
    if len(sys.argv) > 4:
        valu, _ = per_launch(sys.argv[4], "SQ_ACTIVE_INST_VALU")
        insts, _ = per_launch(sys.argv[4], "SQ_INSTS_VALU")
        busy_dir = sys.argv[5] if len(sys.argv) > 5 else sys.argv[4]
        gui, _ = per_launch(busy_dir, "GRBM_GUI_ACTIVE")
        # GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles; 1024 SIMDs (256 CUs x 4)
        cycles = gui / 8.0
        out["valu_insts_per_launch"] = insts
        out["valu_busy"] = valu * 4.0 / (cycles * 1024.0)
        out["valu_note"] = ("SQ_ACTIVE_INST_VALU x 4 / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs); "
                            "the kernel is binary64/binary32 VALU-issue bound, see DESIGN.md")
    with open(sys.argv[3], "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
