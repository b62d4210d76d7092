# A/B of two probe builds (PROBE_BIN_A, PROBE_BIN_B) on C5 knots at full load
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05ab}
mkdir -p $O
for k in 1 20 49 99; do
  for v in A B; do
    bin=PROBE_BIN_$v
    PROBE_BIN=${!bin} PROBE_NT=512 timeout -k 10 60 python tools/mb_probe.py C5_talos_walk $k 2048 > $O/probe_${v}_$k.log 2>&1 || { tail $O/probe_${v}_$k.log; exit 1; }
  done
done
