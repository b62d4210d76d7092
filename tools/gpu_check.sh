# GPU check: GPU suite (parity errors logged to $O/parity.jsonl; MEASURE=1 logs every bar
# without asserting), smoke, the phase-by-phase parity trace (TRACE=1), the 2-rank
# rehearsal of the sharded job on the 1-GPU lease (DIST=1), the C5 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r06}
mkdir -p $O
export CROCODDYL_AMD_PARITY_LOG=$PWD/$O/parity.jsonl
rm -f $CROCODDYL_AMD_PARITY_LOG
if [ -z "$NO_TESTS" ]; then
  CROCODDYL_AMD_PARITY_MEASURE=${MEASURE:-0} timeout -k 10 900 python -u -m pytest -x -v --timeout 200 \
    --timeout-method thread tests -m gpu ${TESTS_K:+-k "$TESTS_K"} > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
  tail -3 $O/gpu_tests.log
fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ -n "$TRACE" ]; then
  timeout -k 10 300 python -u tools/parity_trace.py C5_talos_walk 8 3 3 ${REPS:-3} > $O/parity_trace.log 2>&1 || { tail -5 $O/parity_trace.log; exit 1; }
fi
if [ -n "$DIST" ]; then
  timeout -k 10 400 python -u bench.py --gpus 2 --rehearsal --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_gpus2.json 2> $O/bench_gpus2.err || { tail -20 $O/bench_gpus2.err; exit 1; }
fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > $O/bench_c5.json 2> $O/bench_c5.err || { tail -5 $O/bench_c5.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_c5.json'));print(d['value'],d['kernel_ms_per_step'],d['secondary_protocol'] and d['secondary_protocol']['value'])"
fi
