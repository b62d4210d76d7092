# round 2 counters on the C5 bench: MFMA / busy cycles, then HBM bytes (separate passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
L=gpurun_out/prof/counters.txt
timeout -s KILL 120 rocprofv3 -L > $L 2>&1 || exit 1
pick() { for c in "$@"; do grep -qw "$c" $L && printf "%s " "$c"; done; return 0; }
C1=$(pick SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE)
echo "pass 1 counters: $C1"
timeout -s KILL 240 rocprofv3 --pmc $C1 --output-format csv -d gpurun_out/prof/pmc_mfma -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/pmc_mfma.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/pmc_write.log 2>&1 || exit 1
find gpurun_out/prof -name "*counter_collection*"
