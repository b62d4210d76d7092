"""Per-step kernel times from a rocprofv3 kernel trace, restricted to the last K solves.

bench.py's step is one solve of every element; every solve starts with exactly one
init_state_kernel launch. This tool splits the trace at those launches, keeps the last
K steps (the timed region when the trace is of `bench.py --steps K`), and reports per
kernel class the mean device time per step and per launch — in the units of bench.py's
`rooflines` (calcDiff = the knot-parallel calc + calcDiff kernel and the gaps pass,
backward = the Riccati sweep, forward = one line search: every trial-group launch and
ls_select of the step).

usage: python tools/trace_window.py TRACE_CSV STEPS [OUT_JSON]
"""
import csv
import json
import statistics
import sys

CLASSES = {
    "calcDiff": ("mb_knot_kernel", "calc_diff_kernel", "calc_tiled_kernel", "cost_sum_kernel"),
    "backward": ("backward_mfma_kernel", "backward_kernel"),
    "forward": ("forward_kernel", "ls_select_kernel"),
}


def classify(name):
    for k, subs in CLASSES.items():
        if any(s in name for s in subs):
            return k
    return "other"


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name") or r.get("Name") or ""
            t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            rows.append((t0, t1, name))
    rows.sort()
    starts = [i for i, (_, _, n) in enumerate(rows) if "init_state_kernel" in n]
    if len(starts) < steps:
        raise SystemExit(f"only {len(starts)} solves in the trace, {steps} asked")
    first = starts[-steps]
    win = rows[first:]
    per_step = {}
    launches = {}
    bounds = starts[-steps:] + [len(rows)]
    for s in range(steps):
        for t0, t1, n in rows[bounds[s]:bounds[s + 1]]:
            c = classify(n)
            per_step.setdefault(c, [0.0] * steps)[s] += (t1 - t0) * 1e-6
            key = n.split("(")[0]
            launches.setdefault(key, []).append((t1 - t0) * 1e-6)
    span = (win[-1][1] - win[0][0]) * 1e-6
    out = {
        "trace": path, "steps": steps, "window_ms": round(span, 3), "ms_per_step_wall": round(span / steps, 3),
        "class_ms_per_step": {c: round(statistics.mean(v), 3) for c, v in per_step.items()},
        "kernels": {k: {"launches_per_step": round(len(v) / steps, 2), "mean_ms": round(statistics.mean(v), 4),
                        "total_ms_per_step": round(sum(v) / steps, 3)} for k, v in sorted(launches.items())},
    }
    print(json.dumps(out, indent=1))
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
