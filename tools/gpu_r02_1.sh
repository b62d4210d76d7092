set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gaits_gpu.py tests/test_freeflyer_gpu.py tests/test_contact_gpu.py > gpurun_out/r02_gait_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r02_gait_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r02_bench_c5walk.json 2> gpurun_out/r02_bench_c5walk.err && tail -c 3000 gpurun_out/r02_bench_c5walk.json &&
timeout -k 10 300 python bench.py --config C4_solo12_trot --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r02_bench_c4trot.json 2> gpurun_out/r02_bench_c4trot.err && tail -c 3000 gpurun_out/r02_bench_c4trot.json
