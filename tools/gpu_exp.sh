# experiment: alternative library variants (lib name suffix as $1), parity subset + bench + stamps
set -o pipefail
mkdir -p gpurun_out
V=$1
export CROCODDYL_AMD_LIB=$PWD/crocoddyl_amd/lib/libfddp_hip_$V.so
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_box_gpu.py -x -q -k "default" --timeout 120 --timeout-method thread > gpurun_out/pytest_$V.log 2>&1 || { tail -30 gpurun_out/pytest_$V.log; exit 1; }
tail -1 gpurun_out/pytest_$V.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_$V.log 2>&1 || { tail -20 gpurun_out/bench_$V.log; exit 1; }
tail -1 gpurun_out/bench_$V.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$V', d['value'], d['ms_per_step'], d['kernel_ms_per_step'], d['roofline']['frac'])"
CROCODDYL_AMD_LIB=$PWD/crocoddyl_amd/lib/libfddp_hip_${V}_stamps.so FDDP_STAMPS=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/stamps_$V.log 2>&1 || { tail -20 gpurun_out/stamps_$V.log; exit 1; }
grep -A9 "fddp stamps. mean" gpurun_out/stamps_$V.log
