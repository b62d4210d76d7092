# round 2 (session 3): SolverBoxFDDP on the real C5 walk (controls boxed at the model limits) vs FDDP
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r02_22
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --solver boxfddp --steps 5 --warmup 1 --no-cpu-baseline > $O/c5_box.json 2> $O/c5_box.err || exit 1
python -c "import json;d=json.load(open('$O/c5_box.json'));print('c5 boxfddp',d['value'],d['kernel_ms_per_step'])"
