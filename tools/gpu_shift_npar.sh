# the shift protocol's rollout against the trial-group size: adaptive (default), then
# CROCODDYL_AMD_LS_PAR = 1, 2, 4, 10
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05sh}
rm -rf $O; mkdir -p $O
A="--protocol shift --steps 5 --warmup 1 --no-cpu-baseline --secondary-steps 0"
timeout -k 10 300 python3 bench.py $A > $O/ad.json 2> $O/ad.err || { tail -5 $O/ad.err; exit 1; }
for p in ${PARS:-1 2 4 10}; do
  CROCODDYL_AMD_LS_PAR=$p timeout -k 10 300 python3 bench.py $A > $O/p$p.json 2> $O/p$p.err || { tail -5 $O/p$p.err; exit 1; }
done
