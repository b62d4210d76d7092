# round 2 (session 3): cost table one record per lane: probe, full GPU suite, C5 + C4 benches, then C3 benches and the closing profiles
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_21
mkdir -p $O
export TMPDIR=/tmp
(timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 1 && PROBE_DIFF_NOCOST=1 timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 1) > $O/probe.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 240 --timeout-method thread tests > $O/gpu_tests.log 2>&1
rc=$?; tail -n 2 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
B="python bench.py --steps 5 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 $B > $O/c5.json 2> $O/c5.err || exit 1
timeout -k 10 300 $B --config C4_solo12_trot > $O/c4.json 2> $O/c4.err || exit 1
for f in c5 c4; do python -c "import json,sys;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['kernel_ms_per_step'])"; done
bash tools/gpu_r02_20.sh
