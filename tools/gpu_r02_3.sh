# round 2: C5 / C4 benches with the free-flyer CPU baseline + kernel-trace stats of C5
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02_3
export TMPDIR=/tmp
timeout -k 10 420 python bench.py --steps 10 --warmup 2 > gpurun_out/r02_3/bench_c5.json 2> gpurun_out/r02_3/bench_c5.err || exit 1
tail -c 600 gpurun_out/r02_3/bench_c5.json
timeout -k 10 300 python bench.py --config C4_solo12_trot --steps 10 --warmup 2 > gpurun_out/r02_3/bench_c4.json 2> gpurun_out/r02_3/bench_c4.err || exit 1
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02_3/kt -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r02_3/kt.log 2>&1 || exit 1
find gpurun_out/r02_3 -name "*stats*"
