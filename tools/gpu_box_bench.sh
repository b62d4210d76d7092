set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_cpp_facade.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_facade.log 2>&1 || { tail -30 gpurun_out/pytest_facade.log; exit 1; }
tail -1 gpurun_out/pytest_facade.log
timeout -k 10 400 python bench.py --solver boxfddp > gpurun_out/bench_box.log 2>&1 || { tail -20 gpurun_out/bench_box.log; exit 1; }
tail -1 gpurun_out/bench_box.log
CROCODDYL_AMD_LIB=$PWD/crocoddyl_amd/lib/libfddp_hip_stamps.so FDDP_STAMPS=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_stamps.log 2>&1 || { tail -20 gpurun_out/bench_stamps.log; exit 1; }
grep -A20 "fddp stamps" gpurun_out/bench_stamps.log
