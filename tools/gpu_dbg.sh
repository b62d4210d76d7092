cd $GRAFT_REPO_ROOT
timeout -k 10 600 python tools/dbg_dir.py > gpurun_out/dbg_dir.log 2>&1; tail -14 gpurun_out/dbg_dir.log
DBG_IT=0 timeout -k 10 600 python tools/dbg_dir.py > gpurun_out/dbg_dir0.log 2>&1; tail -14 gpurun_out/dbg_dir0.log
