# C5 bench only (10 timed steps), fixed protocol, plus the shift protocol's secondary line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05b}
mkdir -p $O
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
