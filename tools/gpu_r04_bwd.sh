# backward change check: broadcast self-check, sweep micro-benchmark, GPU suite, smoke,
# C5 backward stamps, quick C5 / C4 / C3 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04w
mkdir -p $O
timeout -k 10 60 ./tools/permlane_check > $O/permlane.log 2>&1 || { cat $O/permlane.log; exit 1; }
timeout -k 10 60 ./tools/sweep_bench > $O/sweep.log 2>&1 || { cat $O/sweep.log; exit 1; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
CROCODDYL_AMD_LIB=$PWD/crocoddyl_amd/lib/libfddp_hip_stamps.so timeout -k 10 120 python -u tools/diag_stamps.py C5_talos_walk > $O/stamps_c5.log 2>&1 || exit 1
B="python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --secondary-steps 0"
timeout -k 10 300 $B > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
timeout -k 10 300 $B --config C4_solo12_trot > $O/bench_c4.json 2> $O/bench_c4.err || exit 1
timeout -k 10 300 $B --config C3_arm_multibody > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
