# A/B of an environment setting on one config: default, then with $ENVB (e.g. "FDDP_MB_NT=128")
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05env}
rm -rf $O; mkdir -p $O
A="--steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --secondary-steps 0 ${BENCH_ARGS}"
for c in ${CFGS:-C4_solo12_trot}; do
  timeout -k 10 300 python3 bench.py --config $c $A > $O/old_$c.json 2> $O/old_$c.err || { tail -5 $O/old_$c.err; exit 1; }
  env $ENVB timeout -k 10 300 python3 bench.py --config $c $A > $O/new_$c.json 2> $O/new_$c.err || { tail -5 $O/new_$c.err; exit 1; }
done
