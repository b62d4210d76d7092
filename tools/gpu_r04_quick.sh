# quick check: smoke, C5 bench, C5 knot probe (production 512-thread calcDiff; one WG and full load)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 60 ./tools/permlane_check > $O/permlane.log 2>&1 || { cat $O/permlane.log; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --secondary-steps 0 > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
PROBE_NT=512 timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 1 > $O/probe_512_1.log 2>&1 || exit 1
PROBE_NT=512 timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 2048 > $O/probe_512_2048.log 2>&1 || exit 1
if [ -n "$QUICK_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
fi
