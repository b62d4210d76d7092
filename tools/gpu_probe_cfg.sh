# knot-calc / calcDiff phase probe of one config's knot, one workgroup and full load
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05pc}
mkdir -p $O
for nwg in 1 ${NWG:-1024}; do
  PROBE_NT=${PNT:-128} timeout -k 10 60 python tools/mb_probe.py ${CFG:-C3_arm_multibody} ${KNOT:-100} $nwg > $O/probe_$nwg.log 2>&1 || { tail $O/probe_$nwg.log; exit 1; }
done
