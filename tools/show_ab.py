"""Print the kernel times of an A/B directory written by tools/gpu_bwd_ab.sh."""
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "new_*.json"))):
    c = os.path.basename(f)[4:-5]
    for tag in ("old", "new"):
        p = os.path.join(d, f"{tag}_{c}.json")
        if os.path.exists(p):
            j = json.load(open(p))
            print(f"{c:18s} {tag} {j['value']:>11.1f} it/s  {j['kernel_ms_per_step']}")
