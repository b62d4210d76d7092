# round 3: the small-tree configs (C3 free / contact, C4 trot) with the CPU baseline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03s
mkdir -p $O
export TMPDIR=/tmp
for cfg in ${CFGS:-C3_arm_multibody C3_arm_contact C4_solo12_trot}; do
  timeout -k 10 600 python bench.py --config $cfg --steps 10 --warmup 2 ${BENCH_ARGS} > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { tail -20 $O/bench_$cfg.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d.get('cpu_baseline') or {};print(sys.argv[2], d['value'],d['kernel_ms_per_step'],c.get('value'),c.get('cores'),d.get('vs_cpu'))" $O/bench_$cfg.json $cfg
done
if [ -n "$BOX" ]; then
  timeout -k 10 600 python bench.py --solver boxfddp --steps 10 --warmup 2 --secondary-steps 0 ${BOX_ARGS} > $O/bench_box.json 2> $O/bench_box.err || { tail -20 $O/bench_box.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));c=d.get('cpu_baseline') or {};print('box', d['value'],d['kernel_ms_per_step'],d['line_search_trials_last_step'],c.get('value'))" $O/bench_box.json
fi
