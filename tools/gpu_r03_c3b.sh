# round 3: small-tree calcDiff at 128 threads (probe, multibody GPU tests, C3 / C4 / C5 benches)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c
mkdir -p $O
export TMPDIR=/tmp
PROBE_NT=128 timeout -k 10 60 python tools/mb_probe.py C3_arm_multibody 10 1 > $O/probe128.log 2>&1 || exit 1
PROBE_NT=128 timeout -k 10 60 python tools/mb_probe.py C3_arm_multibody 10 2048 > $O/probe128_2048.log 2>&1 || exit 1
grep -h "nwg 1:\|nwg 2048:\|total" $O/probe128.log $O/probe128_2048.log
timeout -k 10 900 python -u -m pytest tests/test_multibody_gpu.py tests/test_contact_gpu.py tests/test_box_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
CFGS="C3_arm_multibody C3_arm_contact C4_solo12_trot" BENCH_ARGS=--no-cpu-baseline BOX=1 BOX_ARGS=--no-cpu-baseline bash tools/gpu_r03_small.sh || exit 1
python -c "import json;d=json.load(open('gpurun_out/r03s/bench_box.json'));print(d.get('box_backward'))"
