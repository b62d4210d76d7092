# round 3: small-tree (C3) calcDiff probe phases, box-QP backward phase stamps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03c
mkdir -p $O
export TMPDIR=/tmp
for k in "C3_arm_multibody 10" "C3_arm_contact 10" "C4_solo12_trot 10"; do
  set -- $k
  timeout -k 10 60 python tools/mb_probe.py $1 $2 1 > $O/probe_$1.log 2>&1 || exit 1
  timeout -k 10 60 python tools/mb_probe.py $1 $2 2048 > $O/probe_$1_2048.log 2>&1 || exit 1
done
grep -h "nwg 1:\|nwg 2048:\|phases\|total" $O/probe_*.log
L=$PWD/crocoddyl_amd/lib/libfddp_hip_stamps.so
CROCODDYL_AMD_LIB=$L FDDP_STAMPS=1 timeout -k 10 600 python bench.py --solver boxfddp --steps 2 --warmup 1 --no-cpu-baseline > $O/box_stamps.json 2> $O/box_stamps.err || exit 1
CROCODDYL_AMD_LIB=$L FDDP_STAMPS=1 timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --secondary-steps 0 > $O/fddp_stamps.json 2> $O/fddp_stamps.err || exit 1
grep -A12 "fddp stamps" $O/box_stamps.err | tail -14
grep -A12 "fddp stamps" $O/fddp_stamps.err | tail -14
