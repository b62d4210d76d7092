# host-model GPU test, C5 / C4 benches with CPU baselines, C5 kernel trace, then counters
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02_5
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 240 --timeout-method thread tests/test_host_models.py > gpurun_out/r02_5/host_models.log 2>&1
rc=$?; tail -2 gpurun_out/r02_5/host_models.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 420 python bench.py --steps 10 --warmup 2 > gpurun_out/r02_5/bench_c5.json 2> gpurun_out/r02_5/bench_c5.err || exit 1
timeout -k 10 300 python bench.py --config C4_solo12_trot --steps 10 --warmup 2 > gpurun_out/r02_5/bench_c4.json 2> gpurun_out/r02_5/bench_c4.err || exit 1
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02_5/kt -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r02_5/kt.log 2>&1 || exit 1
python -c "import json;d=json.load(open('gpurun_out/r02_5/bench_c5.json'));print(d['value'],d['kernel_ms_per_step'],d.get('speedup_vs_cpu'))"
bash tools/gpu_r02_6.sh
