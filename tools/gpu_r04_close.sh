# closing run: GPU suite, smoke, bench lines with the CPU port (C5 default, C2, C3, C4), C5 + C2 profiles
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04close2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench_c5.json 2> $O/bench_c5.err || { tail -5 $O/bench_c5.err; exit 1; }
for cfg in C2_lqr C3_arm_multibody C4_solo12_trot; do
  timeout -k 10 400 python -u bench.py --config $cfg > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { tail -5 $O/bench_$cfg.err; exit 1; }
done
PROF_TAG=c5 bash tools/prof_r04.sh || exit 1
PROF_TAG=c2 BENCH_ARGS="--config C2_lqr" bash tools/prof_r04.sh || exit 1
