# round 3 GPU run: the GPU suite (test failures do not stop the run; a crash, an abort or
# a time limit does), smoke, the bench in the default (fixed) protocol with the CPU
# baseline, then a rocprofv3 kernel trace of the bench alone.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03
mkdir -p $O
export TMPDIR=/tmp
ok_or_fail() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; echo "pytest rc=$rc"
ok_or_fail $rc || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python bench.py --steps 10 --warmup 2 ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['kernel_ms_per_step'],d['line_search_trials_last_step'],d['secondary_protocol'],d.get('speedup_vs_cpu'),d['cpu_baseline'].get('value'),d['cpu_baseline'].get('error'),d['roofline']['frac'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --secondary-steps 0 ${BENCH_ARGS} > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
python tools/trace_window.py $(find $O/kt -name "run_kernel_trace.csv" | head -1) 5 $O/trace_window.json | tail -15
