# round 3: calcDiff workgroup size A/B (probe phases at 512 threads, tests, bench default vs FDDP_MB_NT=256)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03n
mkdir -p $O
export TMPDIR=/tmp
PROBE_NT=512 timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 1 > $O/probe512.log 2>&1 || exit 1
PROBE_NT=512 timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 2048 > $O/probe512_2048.log 2>&1 || exit 1
grep -h "calcDiff nwg\|total\|phases" $O/probe512.log $O/probe512_2048.log
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_contact_gpu.py tests/test_gaits_gpu.py tests/test_freeflyer_gpu.py} -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest512.log 2>&1
rc=$?; tail -3 $O/pytest512.log; [ $rc -eq 0 ] || exit 1
summ() { python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'],d['kernel_ms_per_step'])" $1 $2; }
timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --secondary-steps 0 > $O/b512.json 2> $O/b512.err || exit 1
summ $O/b512.json default
for ab in $AB; do
  env $ab timeout -k 10 600 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --secondary-steps 0 > $O/bab.json 2> $O/bab.err || exit 1
  summ $O/bab.json "$ab"
done
