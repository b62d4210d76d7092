# bench lines of the other configs (with their CPU baselines)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05cfg}
mkdir -p $O
for c in ${CFGS:-C2_lqr C3_arm_multibody C4_solo12_trot}; do
  timeout -k 10 500 python3 bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 1; }
done
