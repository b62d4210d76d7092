"""Per-kernel register / scratch resources of a built libfddp_hip.so (gfx950 code object).

    python tools/kernel_resources.py crocoddyl_amd/lib/libfddp_hip.so
    python tools/kernel_resources.py --check crocoddyl_amd/csrc/kernel_budget.json LIB
    python tools/kernel_resources.py --write crocoddyl_amd/csrc/kernel_budget.json LIB

Reads the AMDGPU code-object metadata (.vgpr_count, .agpr_count, .vgpr_spill_count,
.sgpr_spill_count, .private_segment_fixed_size = scratch bytes per lane) of every
kernel: the .hip_fatbin sections of the shared object are unbundled with
clang-offload-bundler and their notes read with llvm-readelf (ROCm's llvm). --check
fails (exit 1) when a kernel spills more VGPRs or uses more scratch than the budget
file allows (a kernel absent from the budget must be spill-free); --write records the
current values as the budget. The build runs --check after linking (csrc/Makefile).
"""
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
FIELDS = ("vgpr_count", "agpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size",
          "group_segment_fixed_size")


def _sections(lib):
    """The .hip_fatbin payloads of the shared object: with several objects linked each
    keeps its own bundle, concatenated in the section (each starts with the magic)."""
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", lib, os.path.join(d, "x")],
                       check=True, capture_output=True)
        data = open(fat, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    return [data[s:(starts[i + 1] if i + 1 < len(starts) else len(data))] for i, s in enumerate(starts)]


def kernels(lib):
    """{kernel symbol: {field: value}} over every code object in the library."""
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for i, blob in enumerate(_sections(lib)):
            b = os.path.join(d, f"b{i}.bin")
            co = os.path.join(d, f"co{i}.elf")
            open(b, "wb").write(blob)
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--unbundle", f"--input={b}",
                                f"--output={co}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"],
                               capture_output=True)
            if r.returncode != 0 or not os.path.exists(co) or os.path.getsize(co) == 0:
                continue
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                                   text=True).stdout
            cur = {}
            for line in notes.splitlines():
                # kernel-level keys only: "  - .key:" opens a record, "    .key:" continues it
                m = re.match(r"(  - |    )\.(\w+):\s+(\S+)", line)
                if not m:
                    continue
                k, v = m.group(2), m.group(3)
                if m.group(1) == "  - ":  # a new kernel record begins
                    cur = {}
                if k in FIELDS:
                    cur[k] = int(v)
                if k == "name":
                    cur["name"] = v
                if "name" in cur and all(f in cur for f in FIELDS[:5]):
                    out[cur["name"]] = {f: cur.get(f, 0) for f in FIELDS}
    return out


def demangle(names):
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    except OSError:
        return {n: n for n in names}
    return dict(zip(names, r.stdout.splitlines())) if r.returncode == 0 else {n: n for n in names}


def main(argv):
    mode, budget_path = None, None
    if argv and argv[0] in ("--check", "--write"):
        mode, budget_path = argv[0], argv[1]
        argv = argv[2:]
    lib = argv[0] if argv else os.path.join(os.path.dirname(__file__), "..", "crocoddyl_amd", "lib", "libfddp_hip.so")
    ks = kernels(lib)
    if not ks:
        print(f"kernel_resources: no gfx950 kernels found in {lib}", file=sys.stderr)
        return 1
    dm = demangle(sorted(ks))
    if mode == "--write":
        json.dump({"note": "per-kernel ceilings checked after every build (tools/kernel_resources.py); "
                           "lower them as kernels improve, never raise them silently",
                   "kernels": {n: {"vgpr_spill_count": v["vgpr_spill_count"],
                                   "private_segment_fixed_size": v["private_segment_fixed_size"]}
                               for n, v in sorted(ks.items())}},
                  open(budget_path, "w"), indent=1)
        print(f"wrote {budget_path}: {len(ks)} kernels")
        return 0
    bad = []
    if mode == "--check":
        budget = json.load(open(budget_path))["kernels"]
        for n, v in ks.items():
            b = budget.get(n, {"vgpr_spill_count": 0, "private_segment_fixed_size": 0})
            for f in ("vgpr_spill_count", "private_segment_fixed_size"):
                if v[f] > b[f]:
                    bad.append(f"{dm[n]}: {f} {v[f]} > budget {b[f]}")
    else:
        w = max(len(dm[n]) for n in ks)
        print(f"{'kernel':<{min(w, 90)}} vgpr agpr vspill sspill scratch")
        for n, v in sorted(ks.items(), key=lambda kv: -kv[1]["vgpr_spill_count"] - kv[1]["private_segment_fixed_size"]):
            print(f"{dm[n][:90]:<{min(w, 90)}} {v['vgpr_count']:4d} {v['agpr_count']:4d} {v['vgpr_spill_count']:6d} "
                  f"{v['sgpr_spill_count']:6d} {v['private_segment_fixed_size']:7d}")
    if bad:
        print("kernel_resources: spill / scratch regression:\n  " + "\n  ".join(bad), file=sys.stderr)
        return 1
    if mode == "--check":
        hot = sorted(ks.items(), key=lambda kv: -kv[1]["private_segment_fixed_size"])[:3]
        print("kernel_resources: within budget; largest scratch: " +
              ", ".join(f"{dm[n].split('(')[0]} {v['private_segment_fixed_size']} B / {v['vgpr_spill_count']} VGPR spills"
                        for n, v in hot))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
