# probe only: C5 knot 20 (one WG and full load), the 512-thread calcDiff and the calc
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05p}
mkdir -p $O
PROBE_NT=512 timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 1 > $O/probe_512_1.log 2>&1 || { tail $O/probe_512_1.log; exit 1; }
PROBE_NT=512 timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 2048 > $O/probe_512_2048.log 2>&1 || { tail $O/probe_512_2048.log; exit 1; }
