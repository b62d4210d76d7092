# round 2 (session 3): C3 arm benches (free / contact dynamics) with their CPU baselines, then the closing C5 profiles again
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_20
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --config C3_arm_multibody --steps 10 --warmup 2 > $O/c3_mb.json 2> $O/c3_mb.err || exit 1
timeout -k 10 300 python bench.py --config C3_arm_contact --steps 10 --warmup 2 > $O/c3_contact.json 2> $O/c3_contact.err || exit 1
for f in c3_mb c3_contact; do python -c "import json,sys;d=json.load(open('$O/$f.json'));print('$f',d['value'],d['kernel_ms_per_step'],d.get('speedup_vs_cpu'))"; done
bash tools/gpu_r02_final.sh
