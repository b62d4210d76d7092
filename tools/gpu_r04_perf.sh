# round-4 perf check: GPU tests (multibody / gaits / dense), the smoke, quick benches of
# C5 / C4 / C3 / C2 with the backward-variant A/B, the C5 knot phase probe
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04
mkdir -p $O
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --secondary-steps 0"
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 $B > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
timeout -k 10 300 $B --config C4_solo12_trot > $O/bench_c4.json 2> $O/bench_c4.err || exit 1
FDDP_BWD_WAVES=8 timeout -k 10 300 $B --config C4_solo12_trot > $O/bench_c4_w8.json 2> $O/bench_c4_w8.err || exit 1
timeout -k 10 300 $B --config C3_arm_multibody > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
FDDP_BWD_WAVES=8 timeout -k 10 300 $B --config C3_arm_multibody > $O/bench_c3_w8.json 2> $O/bench_c3_w8.err || exit 1
timeout -k 10 300 $B --config C2_lqr > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
FDDP_BWD_WAVES=8 timeout -k 10 300 $B --config C2_lqr > $O/bench_c2_w8.json 2> $O/bench_c2_w8.err || exit 1
for k in 20 1; do timeout -k 10 60 python tools/mb_probe.py C5_talos_walk $k 1 > $O/probe_$k.log 2>&1 || exit 1; done
