# round-5 GPU check: GPU suite (parity errors logged to $O/parity.jsonl; MEASURE=1 logs
# every bar without asserting), smoke, the 2-rank launcher on the 1-GPU lease, the C5 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05}
mkdir -p $O
export CROCODDYL_AMD_PARITY_LOG=$PWD/$O/parity.jsonl
rm -f $CROCODDYL_AMD_PARITY_LOG
if [ -z "$NO_TESTS" ]; then
  CROCODDYL_AMD_PARITY_MEASURE=${MEASURE:-0} timeout -k 10 900 python -u -m pytest -x -v --timeout 200 \
    --timeout-method thread tests -m gpu ${TESTS_K:+-k "$TESTS_K"} > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
fi
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
if [ -z "$NO_DIST" ]; then
  timeout -k 10 400 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_gpus2.json 2> $O/bench_gpus2.err || { tail -20 $O/bench_gpus2.err; exit 1; }
fi
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > $O/bench_c5.json 2> $O/bench_c5.err || { tail -5 $O/bench_c5.err; exit 1; }
