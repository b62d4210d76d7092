cd $GRAFT_REPO_ROOT
TESTS="tests/test_fullsize_gpu.py tests/test_gaits_gpu.py tests/test_contact_gpu.py tests/test_multibody_gpu.py tests/test_freeflyer_gpu.py" bash tools/gpu_r03_iter.sh || exit 1
timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 1 > gpurun_out/r03i/probe_c5_20.log 2>&1 || exit 1
timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 2048 > gpurun_out/r03i/probe_c5_20_2048.log 2>&1 || exit 1
tail -12 gpurun_out/r03i/probe_c5_20.log
