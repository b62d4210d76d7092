# quick check: labelled probe (C5 knot 20) and the C5 bench (10 steps)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05q}
mkdir -p $O
timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 2048 > $O/probe_tree.log 2>&1 || { tail $O/probe_tree.log; exit 1; }
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --secondary-steps 0 ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
