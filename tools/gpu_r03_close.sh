# round 3 closing run: the GPU suite, smoke, the C5 bench with the CPU baseline, then the
# rocprofv3 kernel trace and counter passes of the bench (tools/prof_r03.sh)
bash tools/gpu_r03_run.sh || exit 1
bash tools/prof_r03.sh || exit 1
