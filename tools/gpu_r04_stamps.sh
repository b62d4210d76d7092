# backward-sweep phase stamps (C5 / C4 / C3): this tree vs the round-3 tree in _r3/
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04s
mkdir -p $O
for cfg in C5_talos_walk C4_solo12_trot C3_arm_multibody; do
  FDDP_BWD_WAVES=8 CROCODDYL_AMD_LIB=$PWD/crocoddyl_amd/lib/libfddp_hip_stamps.so timeout -k 10 120 python -u tools/diag_stamps.py $cfg > $O/now_$cfg.log 2>&1 || exit 1
  (cd _r3 && CROCODDYL_AMD_LIB=$PWD/crocoddyl_amd/lib/libfddp_hip_stamps.so timeout -k 10 120 python -u tools/diag_stamps.py $cfg) > $O/r3_$cfg.log 2>&1 || exit 1
done
