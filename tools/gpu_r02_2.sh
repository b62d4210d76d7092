set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_probe.sh > gpurun_out/probe6.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gaits_gpu.py tests/test_freeflyer_gpu.py tests/test_contact_gpu.py tests/test_multibody_gpu.py > gpurun_out/r02_mb_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r02_mb_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r02_bench_c5walk.json 2> gpurun_out/r02_bench_c5walk.err && python -c "import json;d=json.load(open('gpurun_out/r02_bench_c5walk.json'));print(d['value'],d['kernel_ms_per_step'])"
