# round 3 iteration run: selected GPU tests (TESTS), then the bench without the CPU
# baseline, plus optional A/B env settings (AB="VAR=val ...", one bench each).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03i
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -4 $O/pytest.log; echo "pytest rc=$rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
fi
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'],d['kernel_ms_per_step'],d['line_search_trials_last_step']['hist'],(d.get('secondary_protocol') or {}).get('value'))" $1 $2; }
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
summ $O/bench.json default
i=0
for ab in $AB; do
  i=$((i+1))
  env $ab timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --secondary-steps 0 ${BENCH_ARGS} > $O/bench_ab$i.json 2> $O/bench_ab$i.err || { tail -20 $O/bench_ab$i.err; exit 1; }
  summ $O/bench_ab$i.json "$ab"
done
