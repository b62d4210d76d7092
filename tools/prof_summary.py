"""Summarise a rocprofv3 profiling run (tools/prof.sh) into profiles/.

Inputs (gpurun_out/prof/...):
  kt/run_kernel_stats.csv            rocprofv3 --kernel-trace --stats
  pmc_fetch/run_counter_collection.csv   rocprofv3 --pmc FETCH_SIZE
  pmc_write/run_counter_collection.csv   rocprofv3 --pmc WRITE_SIZE
Outputs:
  profiles/<tag>_kernel_stats.csv    (copy)
  profiles/pmc_backward.json         HBM bytes per backward launch, as bench.py's roofline "traffic"

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. On gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md, HBM
section): it is doubled here; WRITE_SIZE is taken as is.
"""
import csv
import glob
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counter(path, name_sub, counter_name):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if name_sub in row["Kernel_Name"] and row["Counter_Name"] == counter_name:
                vals.append(float(row["Counter_Value"]))
    return vals


def find(d, name):
    """rocprofv3 writes under <dir>/<host>/<pid>/ or straight into <dir>."""
    hits = sorted(glob.glob(os.path.join(d, "**", name), recursive=True))
    return hits[0] if hits else os.path.join(d, name)


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    cfg = sys.argv[2] if len(sys.argv) > 2 else "C5_talos_full"
    src = os.path.join(ROOT, "gpurun_out", "prof")
    kt = sys.argv[3] if len(sys.argv) > 3 else os.path.join(src, "kt")
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(find(kt, "run_kernel_stats.csv"), os.path.join(prof, f"{tag}_kernel_stats.csv"))
    out = {}
    for kname, key in (("backward_mfma_kernel", "backward"), ("calc_fused_kernel", "calc_fused"),
                       ("forward_kernel", "forward"), ("mb_knot_kernel", "mb_calc_diff")):
        f = counter(find(os.path.join(src, "pmc_fetch"), "run_counter_collection.csv"), kname, "FETCH_SIZE")
        w = counter(find(os.path.join(src, "pmc_write"), "run_counter_collection.csv"), kname, "WRITE_SIZE")
        if not f or not w:
            continue
        # steady state: drop the first (cold) dispatch when there are several
        f = f[1:] if len(f) > 2 else f
        w = w[1:] if len(w) > 2 else w
        fetch = 2.0 * statistics.mean(f) * 1024.0
        write = statistics.mean(w) * 1024.0
        out[key] = {"hbm_bytes_per_launch": fetch + write, "fetch_bytes": fetch, "write_bytes": write,
                    "dispatches": [len(f), len(w)]}
        mf = find(os.path.join(src, "pmc_mfma"), "run_counter_collection.csv")
        if os.path.exists(mf):  # MFMA / busy counters (SQ_* summed over the SIMDs, GRBM over the 8 XCDs)
            c = {n: statistics.mean(counter(mf, kname, n) or [0.]) for n in
                 ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU_MFMA_F64", "SQ_INSTS_VALU_MFMA_MOPS_F64",
                  "SQ_INSTS_VALU", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE")}
            clk = c["GRBM_GUI_ACTIVE"] / 8.0  # per-XCD GPU cycles of the dispatch
            c["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / max(clk * 256 * 4, 1.0)  # per SIMD
            c["mfma_f64_flops"] = c["SQ_INSTS_VALU_MFMA_F64"] * 16 * 16 * 4 * 2  # v_mfma_f64_16x16x4
            out[key]["counters"] = c
    path = os.path.join(prof, "pmc_backward.json")
    data = json.load(open(path)) if os.path.exists(path) else {}
    data[cfg] = dict(out.get("backward", {}), kernels=out, tag=tag,
                     note="FETCH_SIZE x2 (gfx950 streaming-read correction) + WRITE_SIZE, KiB -> bytes, "
                          "mean over steady-state dispatches")
    json.dump(data, open(path, "w"), indent=1)
    print(json.dumps(data[cfg], indent=1))


if __name__ == "__main__":
    main()
