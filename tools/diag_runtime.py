"""Diagnostic (not a test): which HIP runtime the process binds, in both import orders."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
mode = sys.argv[1] if len(sys.argv) > 1 else "none"
if mode == "torch_first":
    import torch
    print("torch", torch.__version__, torch.cuda.is_available(), torch.version.hip)
import helpers  # noqa: E402

S = helpers.setup("C2_lqr", T=4, B=2)
g = helpers.Gpu(S["dims"], S["knots"], S["pool"], S["x0s"])
g.set_candidate(None, None, False)
r = g.solve(10)
print("solve ok", [x.iter for x in r], [x.cost for x in r])
if mode == "lib_first":
    import torch
    print("torch after", torch.cuda.is_available(), torch.zeros(3, device="cuda").sum().item())
with open("/proc/self/maps") as f:
    print(sorted(set(ln.split()[-1] for ln in f if "amdhip" in ln or "hsa-runtime" in ln)))
