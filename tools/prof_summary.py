"""Summarise a rocprofv3 profiling run (tools/prof.sh) into profiles/.

Inputs (gpurun_out/prof/...):
  kt/run_kernel_stats.csv                rocprofv3 --kernel-trace --stats
  pmc_fetch/run_counter_collection.csv   rocprofv3 --pmc FETCH_SIZE
  pmc_write/run_counter_collection.csv   rocprofv3 --pmc WRITE_SIZE
  pmc_mfma/run_counter_collection.csv    rocprofv3 --pmc SQ_* / GRBM_GUI_ACTIVE (optional)
Outputs:
  profiles/<tag>_kernel_stats.csv    (copy)
  profiles/pmc_backward.json[cfg]    per kernel class: HBM bytes per launch and per step

Only the dispatches of the timed steps are kept: bench.py's step is one solve, every
solve starts with one init_state_kernel launch, and the profiled command is
`bench.py --steps K --secondary-steps 0`, so the last K solves are the timed region
(as tools/trace_window.py does for the kernel trace). Per class: the mean per
dispatch and the sum per step (forward: one line search = every trial-group launch
of the step, which is what bench.py's rollout roofline divides by).

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

CLASSES = {  # bench.py's rooflines keys -> kernel name fragments
    "backward": ("backward_mfma_kernel", "backward_kernel"),
    "forward": ("forward_kernel",),
    "mb_calc_diff": ("mb_knot_kernel",),
    "calc_fused": ("calc_tiled_kernel", "calc_diff_kernel"),  # the dense knots' calc / calcDiff
}


def window_rows(path, counter_name, steps):
    """(dispatch name, value) of counter_name for the dispatches of the last `steps`
    solves, grouped per step: [[(name, value), ...] per step]."""
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter_name:
                continue
            rows.append((int(r["Start_Timestamp"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    starts = [i for i, (_, n, _) in enumerate(rows) if "init_state_kernel" in n]
    if len(starts) < steps:
        raise SystemExit(f"{path}: only {len(starts)} solves, {steps} asked")
    bounds = starts[-steps:] + [len(rows)]
    return [[(n, v) for _, n, v in rows[bounds[s]:bounds[s + 1]]] for s in range(steps)]


def class_stats(per_step, subs):
    """mean per dispatch, mean per step, dispatches per step of the kernels matching subs."""
    disp, step_sums, counts = [], [], []
    for st in per_step:
        vals = [v for n, v in st if any(s in n for s in subs)]
        disp += vals
        step_sums.append(sum(vals))
        counts.append(len(vals))
    if not disp:
        return None
    return statistics.mean(disp), statistics.mean(step_sums), statistics.mean(counts)


def find(d, name):
    """rocprofv3 writes under <dir>/<host>/<pid>/ or straight into <dir>."""
    hits = sorted(glob.glob(os.path.join(d, "**", name), recursive=True))
    return hits[0] if hits else os.path.join(d, name)


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r04"
    cfg = sys.argv[2] if len(sys.argv) > 2 else "C5_talos_walk"
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    src = sys.argv[4] if len(sys.argv) > 4 else os.path.join(ROOT, "gpurun_out", "prof")
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    ks = find(os.path.join(src, "kt"), "run_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(prof, f"{tag}_{cfg}_kernel_stats.csv"))
    fetch = window_rows(find(os.path.join(src, "pmc_fetch"), "run_counter_collection.csv"), "FETCH_SIZE", steps)
    write = window_rows(find(os.path.join(src, "pmc_write"), "run_counter_collection.csv"), "WRITE_SIZE", steps)
    mf = find(os.path.join(src, "pmc_mfma"), "run_counter_collection.csv")
    out = {}
    for key, subs in CLASSES.items():
        f, w = class_stats(fetch, subs), class_stats(write, subs)
        if not f or not w:
            continue
        kib = 1024.0
        d = {"hbm_bytes_per_launch": (2.0 * f[0] + w[0]) * kib, "fetch_bytes_per_launch": 2.0 * f[0] * kib,
             "write_bytes_per_launch": w[0] * kib, "hbm_bytes_per_step": (2.0 * f[1] + w[1]) * kib,
             "launches_per_step": f[2]}
        if os.path.exists(mf):  # MFMA / busy counters (SQ_* summed over the SIMDs, GRBM over the 8 XCDs)
            c = {}
            for n in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU_MFMA_F64", "SQ_INSTS_VALU_MFMA_MOPS_F64",
                      "SQ_INSTS_VALU", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE"):
                try:
                    s = class_stats(window_rows(mf, n, steps), subs)
                except SystemExit:
                    s = None
                c[n] = s[0] if s else 0.0
            clk = c["GRBM_GUI_ACTIVE"] / 8.0  # per-XCD GPU cycles of the dispatch
            c["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / max(clk * 256 * 4, 1.0)  # per SIMD
            # mean resident waves per CU over the dispatch (SQ_WAVE_CYCLES counts quad-cycles,
            # MI355X_MICROARCH.md; the per-XCD clock as above)
            c["resident_waves_per_cu"] = 4.0 * c["SQ_WAVE_CYCLES"] / max(clk * 256, 1.0)
            c["mfma_f64_flops"] = c["SQ_INSTS_VALU_MFMA_F64"] * 16 * 16 * 4 * 2  # v_mfma_f64_16x16x4
            d["counters"] = c
        out[key] = d
    # the library build the counters belong to: the lib_sha256 of the profiled bench runs'
    # own JSON lines (bench.py uses the entry only when its running library has that hash)
    hashes = set()
    for log in glob.glob(os.path.join(src, "*.json")) + glob.glob(os.path.join(src, "pmc_*.log")):
        for line in open(log, errors="replace"):
            if line.startswith("{") and '"lib_sha256"' in line:
                hashes.add(json.loads(line)["lib_sha256"])
    if len(hashes) != 1:
        raise SystemExit(f"prof_summary: expected one library hash over the profiled runs, found {sorted(hashes)}")
    path = os.path.join(prof, "pmc_backward.json")
    data = json.load(open(path)) if os.path.exists(path) else {}
    data[cfg] = dict(out.get("backward", {}), kernels=out, tag=tag, steps=steps, lib_sha256=hashes.pop(),
                     note="dispatches of the last `steps` solves only (the timed steps); FETCH_SIZE x2 (gfx950 "
                          "streaming-read correction) + WRITE_SIZE, KiB -> bytes; per launch = mean per dispatch, "
                          "per step = sum over the step's dispatches")
    json.dump(data, open(path, "w"), indent=1)
    print(json.dumps(data[cfg], indent=1))


if __name__ == "__main__":
    main()
