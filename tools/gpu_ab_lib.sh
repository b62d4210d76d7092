# A/B of two library builds on the C5 bench (B = the variant at $LIB_B), plus the HBM
# counters of the variant (FETCH_SIZE / WRITE_SIZE passes of 2 timed steps)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05ab}
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --secondary-steps 0 > $O/bench_a.json 2> $O/bench_a.err || { tail -5 $O/bench_a.err; exit 1; }
CROCODDYL_AMD_LIB=$PWD/$LIB_B timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --secondary-steps 0 > $O/bench_b.json 2> $O/bench_b.err || { tail -5 $O/bench_b.err; exit 1; }
PARGS="--steps 2 --warmup 1 --no-cpu-baseline --secondary-steps 0"
CROCODDYL_AMD_LIB=$PWD/$LIB_B timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py $PARGS > $O/pmc_fetch.log 2>&1 || { tail -5 $O/pmc_fetch.log; exit 1; }
CROCODDYL_AMD_LIB=$PWD/$LIB_B timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py $PARGS > $O/pmc_write.log 2>&1 || { tail -5 $O/pmc_write.log; exit 1; }
