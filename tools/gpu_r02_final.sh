# round 2 (session 3) closing measurements on the default C5 bench: the bench line with the
# CPU baseline, a rocprofv3 kernel trace, then MFMA / busy and HBM counters in separate passes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/prof
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 420 python bench.py --steps 10 --warmup 2 > gpurun_out/r02_final_bench.json 2> gpurun_out/r02_final_bench.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/r02_final_bench.json'));print(d['value'],d['kernel_ms_per_step'],d.get('speedup_vs_cpu'))"
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/kt.log 2>&1 || exit 1
L=$O/counters.txt
timeout -s KILL 120 rocprofv3 -L > $L 2>&1 || exit 1
pick() { for c in "$@"; do grep -qw "$c" $L && printf "%s " "$c"; done; return 0; }
C1=$(pick SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE)
echo "pass 1 counters: $C1"
timeout -s KILL 240 rocprofv3 --pmc $C1 --output-format csv -d $O/pmc_mfma -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_mfma.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_write.log 2>&1 || exit 1
find $O -name "*.csv" | head -20
