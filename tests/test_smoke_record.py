"""Regression guard on the headline parity, on the CPU: the newest committed smoke record
(profiles/r<NN>_*_smoke.log, the output of __graft_entry__.smoke() on the MI355X: the C5
Talos walk at T = 8 through the C ABI against the C++ oracle) must keep the state error
after three FDDP iterations within 2x the oracle's own spread under one-ulp parameter
noise (round 5's smoke drifted to 2.5x unnoticed behind a 4x bar), and every reported
quantity within the smoke's own bar max(1e-8, 2 x floor)."""
import glob
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _latest_record():
    logs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_smoke.log")))
    assert logs, "no committed smoke record under profiles/"
    # round tag first (r06 > r05), then the session letter / version
    return logs[-1]


def test_latest_smoke_record_within_twice_the_floor():
    path = _latest_record()
    text = open(path).read()
    line = [ln for ln in text.splitlines() if ln.startswith("smoke ok")]
    assert line, f"{path}: no 'smoke ok' line"
    vals = dict((k, (float(e), float(f))) for k, e, f in re.findall(r"(\w+@\d) ([0-9.e+-]+) \(([0-9.e+-]+)\)", line[-1]))
    assert {"xs@1", "us@1", "cost@1", "xs@3", "us@3", "cost@3"} <= set(vals), vals
    e, fl = vals["xs@3"]
    assert e <= 2.0 * fl, f"{os.path.basename(path)}: smoke xs@3 {e:.3g} > 2 x floor {fl:.3g}"
    for k, (e, fl) in vals.items():
        assert e <= max(1e-8, 2.0 * fl), (os.path.basename(path), k, e, fl)
