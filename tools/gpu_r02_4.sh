# parallel line search: parity tests, the sharded-path test, C5 / C4 with 1 vs 4 trials per group
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02_4
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gaits_gpu.py tests/test_freeflyer_gpu.py tests/test_contact_gpu.py tests/test_multibody_gpu.py tests/test_dist_gpu.py > gpurun_out/r02_4/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r02_4/tests.log; [ $rc -ne 0 ] && exit $rc
for cfg in C5_talos_walk C4_solo12_trot; do
  for par in 1 2 4; do
    CROCODDYL_AMD_LS_PAR=$par timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02_4/bench_${cfg}_par$par.json 2> gpurun_out/r02_4/bench_${cfg}_par$par.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r02_4/bench_${cfg}_par$par.json'));print('$cfg', $par, d['value'], d['kernel_ms_per_step'])"
  done
done
