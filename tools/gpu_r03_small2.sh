# round 3: GPU tests of the multibody paths, then the small-tree benches (no CPU leg) and the box bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gaits_gpu.py tests/test_contact_gpu.py tests/test_multibody_gpu.py tests/test_freeflyer_gpu.py tests/test_box_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit 1
BENCH_ARGS="--no-cpu-baseline" bash tools/gpu_r03_small.sh
