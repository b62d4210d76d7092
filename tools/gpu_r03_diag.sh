# round 3, first box call: CPU-side diagnosis of the -march=native oracle crash (no GPU
# use), then the GPU suite, smoke and the bench in both protocols.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03
O=gpurun_out/r03
echo | gcc -march=native -E -v - 2>&1 | grep cc1 > $O/native_flags.txt
gcc -march=native -Q --help=target 2>/dev/null | grep -E "^  -m(arch|tune|avx|prefer)" >> $O/native_flags.txt
nproc > $O/cpus.txt; cat /sys/fs/cgroup/cpu.max >> $O/cpus.txt 2>&1; ulimit -s >> $O/cpus.txt; grep -m1 "model name" /proc/cpuinfo >> $O/cpus.txt
timeout -k 10 120 python tools/dump_problem.py C5_talos_walk 32 /tmp/c5.bin > $O/dump.log 2>&1 || exit 1
timeout -k 10 300 make -s -C oracle driver OUT=/tmp/drvn ARCH=-march=native > $O/driver_build.log 2>&1 || exit 1
timeout -k 10 300 /tmp/drvn/cpu_driver /tmp/c5.bin 16 2 > $O/driver_native.log 2>&1; echo "native driver exit $?" >> $O/driver_native.log
timeout -k 10 300 /tmp/drvn/cpu_driver /tmp/c5.bin 1 1 > $O/driver_native_1t.log 2>&1; echo "native driver 1 thread exit $?" >> $O/driver_native_1t.log
grep -q "exit 0" $O/driver_native.log || { for a in $(grep -o '\[0x[0-9a-f]*\]' $O/driver_native.log | tr -d '[]' | head -20); do addr2line -f -C -e /tmp/drvn/cpu_driver $a; done > $O/driver_native_addr2line.txt 2>&1; }
cat $O/driver_native.log | tail -5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > $O/bench_fixed.json 2> $O/bench_fixed.err || { tail -20 $O/bench_fixed.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_fixed.json'));print(d['value'],d['kernel_ms_per_step'],d['line_search_trials_last_step'],d['secondary_protocol'],d.get('speedup_vs_cpu'),d['cpu_baseline'].get('value'),d['cpu_baseline'].get('error'))"
