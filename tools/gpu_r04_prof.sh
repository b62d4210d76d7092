# round-4 profiles: C5 (headline) and C2 (LQR 24/12) kernel traces of the timed steps + PMC passes
set -o pipefail
cd $GRAFT_REPO_ROOT
PROF_TAG=c5 bash tools/prof_r04.sh || exit 1
PROF_TAG=c2 BENCH_ARGS="--config C2_lqr" bash tools/prof_r04.sh || exit 1
