# LDS pivot-row Gauss-Jordan in calcDiff: phase probe, parity tests, C5 / C4 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02_8
bash tools/gpu_probe.sh > gpurun_out/r02_8/probe.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gaits_gpu.py tests/test_freeflyer_gpu.py tests/test_contact_gpu.py tests/test_multibody_gpu.py > gpurun_out/r02_8/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r02_8/tests.log; [ $rc -ne 0 ] && exit $rc
for cfg in C5_talos_walk C4_solo12_trot; do
  timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02_8/bench_$cfg.json 2> gpurun_out/r02_8/bench_$cfg.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r02_8/bench_$cfg.json'));print('$cfg', d['value'], d['kernel_ms_per_step'])"
done
