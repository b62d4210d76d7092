# backward-sweep A/B over the configs: the in-tree library (new) against $LIB_B (old),
# kernel times from the bench lines (no CPU baseline); then the backward GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05bab}
rm -rf $O; mkdir -p $O
for c in ${CFGS:-C2_lqr C3_arm_multibody C4_solo12_trot C5_talos_walk}; do
  timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --secondary-steps 0 > $O/new_$c.json 2> $O/new_$c.err || { tail -5 $O/new_$c.err; exit 1; }
  CROCODDYL_AMD_LIB=$PWD/$LIB_B timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --secondary-steps 0 > $O/old_$c.json 2> $O/old_$c.err || { tail -5 $O/old_$c.err; exit 1; }
done
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu ${TESTS_K:+-k "$TESTS_K"} > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
fi
