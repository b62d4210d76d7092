# spilled calcDiff plan: probe (C5 knot 0 = double support and 20, 2 WGs / CU, and the
# all-LDS plan for comparison), the GPU suite, smoke, C5 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05s}
mkdir -p $O
export CROCODDYL_AMD_PARITY_LOG=$PWD/$O/parity.jsonl
rm -f $CROCODDYL_AMD_PARITY_LOG
for k in 0 20; do
  timeout -k 10 60 python tools/mb_probe.py C5_talos_walk $k 2048 > $O/probe_s_${k}.log 2>&1 || { tail $O/probe_s_${k}.log; exit 1; }
done
PROBE_SPILL=0 PROBE_NT=512 timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 2048 > $O/probe_lds512_20.log 2>&1 || { tail $O/probe_lds512_20.log; exit 1; }
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu ${TESTS_K:+-k "$TESTS_K"} > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > $O/bench_c5.json 2> $O/bench_c5.err || { tail -5 $O/bench_c5.err; exit 1; }
FDDP_MB_SPILL=0 timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > $O/bench_c5_lds.json 2> $O/bench_c5_lds.err || { tail -5 $O/bench_c5_lds.err; exit 1; }
