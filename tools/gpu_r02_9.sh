# A/B: calcDiff Gauss-Jordan pivot row by readlane (A) or LDS broadcast (B)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02_9
for v in A B; do
  for cfg in C5_talos_walk C4_solo12_trot; do
    CROCODDYL_AMD_LIB=$GRAFT_REPO_ROOT/crocoddyl_amd/lib/libfddp_hip_$v.so timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02_9/bench_${cfg}_$v.json 2> gpurun_out/r02_9/bench_${cfg}_$v.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/r02_9/bench_${cfg}_$v.json'));print('$v $cfg', d['value'], d['kernel_ms_per_step'])"
  done
done
