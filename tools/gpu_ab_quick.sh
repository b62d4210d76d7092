# quick A/B of two library builds on the C5 bench (B = the variant at $LIB_B), fixed and shift protocols
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05abq}
rm -rf $O; mkdir -p $O
A="--steps 10 --warmup 2 --no-cpu-baseline --secondary-steps ${SEC:-0} ${BENCH_ARGS}"
timeout -k 10 300 python3 bench.py $A > $O/bench_a.json 2> $O/bench_a.err || { tail -5 $O/bench_a.err; exit 1; }
CROCODDYL_AMD_LIB=$PWD/$LIB_B timeout -k 10 300 python3 bench.py $A > $O/bench_b.json 2> $O/bench_b.err || { tail -5 $O/bench_b.err; exit 1; }
