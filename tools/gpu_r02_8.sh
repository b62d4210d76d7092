# round 2 (session 3): GPU suite, then the C5 rollout A/B (generic vs multibody-only kernel, 2 vs 1 waves/EU)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_8
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 240 --timeout-method thread tests > $O/gpu_tests.log 2>&1
rc=$?; tail -n 2 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
B="python bench.py --steps 5 --warmup 1 --no-cpu-baseline"
FDDP_FWD_MB=0 timeout -k 10 300 $B > $O/c5_generic.json 2> $O/c5_generic.err || exit 1
timeout -k 10 300 $B > $O/c5_mb.json 2> $O/c5_mb.err || exit 1
CROCODDYL_AMD_LIB=$PWD/crocoddyl_amd/lib/libfddp_hip_wpe1.so timeout -k 10 300 $B > $O/c5_mb_wpe1.json 2> $O/c5_mb_wpe1.err || exit 1
for f in generic mb mb_wpe1; do python -c "import json,sys;d=json.load(open('$O/c5_$f.json'));print('$f',d['value'],d['kernel_ms_per_step'])"; done
