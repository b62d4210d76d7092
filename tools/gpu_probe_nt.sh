# probe: C5 knot 20, the calcDiff at PROBE_NT threads (one WG, full load)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05nt}
mkdir -p $O
for nt in ${NTS:-256}; do
  PROBE_NT=$nt timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 1 > $O/probe_${nt}_1.log 2>&1 || { tail $O/probe_${nt}_1.log; exit 1; }
  PROBE_NT=$nt timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 2048 > $O/probe_${nt}_2048.log 2>&1 || { tail $O/probe_${nt}_2048.log; exit 1; }
done
