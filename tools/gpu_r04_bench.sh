# round-4 bench lines with the CPU baseline: C5 (the default line), C2, C3, C4
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_c5.json 2> $O/bench_c5.err || { tail -5 $O/bench_c5.err; exit 1; }
for cfg in C2_lqr C3_arm_multibody C4_solo12_trot; do
  timeout -k 10 400 python -u bench.py --config $cfg > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { tail -5 $O/bench_$cfg.err; exit 1; }
done
