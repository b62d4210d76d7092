# round-5 closing profile of the C5 bench (fixed protocol): a rocprofv3 kernel trace of
# exactly the timed steps (trace_window.py keeps the last STEPS solves), then the HBM
# and MFMA counters in separate --pmc passes (FETCH_SIZE and WRITE_SIZE cannot share
# one). Summarised into profiles/ by tools/prof_summary.py.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/prof${PROF_TAG:+_$PROF_TAG}
rm -rf $O
mkdir -p $O
export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --secondary-steps 0 ${BENCH_ARGS}"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py $ARGS > $O/kt.json 2> $O/kt.log || { tail -5 $O/kt.log; exit 1; }
python tools/trace_window.py $(find $O/kt -name "run_kernel_trace.csv" | head -1) 5 $O/trace_window.json | tail -8
PARGS="--steps 2 --warmup 1 --no-cpu-baseline --secondary-steps 0 ${BENCH_ARGS}"
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py $PARGS > $O/pmc_fetch.log 2>&1 || { tail -5 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py $PARGS > $O/pmc_write.log 2>&1 || { tail -5 $O/pmc_write.log; exit 1; }
timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_mfma -o run -- python3 bench.py $PARGS > $O/pmc_mfma.log 2>&1 || { tail -5 $O/pmc_mfma.log; exit 1; }
find $O -name "*.csv" | head -20
# the bench line with its CPU baseline (the default command), kept beside the profile
timeout -k 10 600 python3 bench.py ${BENCH_ARGS} > $O/bench_with_cpu.json 2> $O/bench_with_cpu.log || { tail -5 $O/bench_with_cpu.log; exit 1; }
