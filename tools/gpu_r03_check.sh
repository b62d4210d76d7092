# round 3: one change on the multibody GPU tests, the C5 probe and the C5 / C4 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03k
mkdir -p $O
export TMPDIR=/tmp
PROBE_NT=512 timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 1 > $O/probe_c5.log 2>&1 || { tail $O/probe_c5.log; exit 1; }
grep "phases\|total" $O/probe_c5.log
timeout -k 10 900 python -u -m pytest tests/test_multibody_gpu.py tests/test_contact_gpu.py tests/test_freeflyer_gpu.py tests/test_gaits_gpu.py tests/test_fullsize_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for cfg in C5_talos_walk C4_solo12_trot; do
  timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --secondary-steps 0 > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { tail -20 $O/bench_$cfg.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], d['value'],d['kernel_ms_per_step'])" $O/bench_$cfg.json $cfg
done
