# tree-LTDL check: probe phases (C5 knot 20, one WG and full load), GPU suite, smoke, C5 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05t}
mkdir -p $O
export CROCODDYL_AMD_PARITY_LOG=$PWD/$O/parity.jsonl
rm -f $CROCODDYL_AMD_PARITY_LOG
PROBE_NT=512 timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 1 > $O/probe_512_1.log 2>&1 || { tail $O/probe_512_1.log; exit 1; }
PROBE_NT=512 timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 2048 > $O/probe_512_2048.log 2>&1 || { tail $O/probe_512_2048.log; exit 1; }
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu ${TESTS_K:+-k "$TESTS_K"} > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > $O/bench_c5.json 2> $O/bench_c5.err || { tail -5 $O/bench_c5.err; exit 1; }
