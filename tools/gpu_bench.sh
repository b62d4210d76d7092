cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err && python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['value'],d['kernel_ms_per_step'],d['line_search_trials_last_step'])"
