# labelled phase probes (C5 knot 20, full load): the calcDiff as the library runs it
# (spilled plan, 2 workgroups / CU) and the calc both ways (tree solve / dense GJ)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05lab2}
mkdir -p $O
timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 2048 > $O/probe_tree.log 2>&1 || { tail $O/probe_tree.log; exit 1; }
PROBE_BIN=$PWD/tools/mb_probe_dense timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 2048 > $O/probe_dense.log 2>&1 || { tail $O/probe_dense.log; exit 1; }
