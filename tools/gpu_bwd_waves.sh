# backward plan A/B: eight-wave (default) against FDDP_BWD_WAVES=$W (four-wave) per config
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05bw}
rm -rf $O; mkdir -p $O
for c in ${CFGS:-C3_arm_multibody C4_solo12_trot C2_lqr}; do
  timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --secondary-steps 0 > $O/old_$c.json 2> $O/old_$c.err || { tail -5 $O/old_$c.err; exit 1; }
  FDDP_BWD_WAVES=${W:-4} timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --secondary-steps 0 > $O/new_$c.json 2> $O/new_$c.err || { tail -5 $O/new_$c.err; exit 1; }
done
