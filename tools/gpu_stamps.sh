# backward-sweep phase stamps (stamps build) for the configs in $CFGS
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05st}
mkdir -p $O
for c in ${CFGS:-C2_lqr}; do
  CROCODDYL_AMD_LIB=$PWD/crocoddyl_amd/lib/libfddp_hip_stamps.so timeout -k 10 200 python3 tools/diag_stamps.py $c > $O/stamps_$c.log 2>&1 || { tail -5 $O/stamps_$c.log; exit 1; }
done
[ -n "$NO_C2" ] || timeout -k 10 300 python3 bench.py --config C2_lqr --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
