cd $GRAFT_REPO_ROOT
for k in 20 1 49; do timeout -k 10 60 python tools/mb_probe.py C5_talos_walk $k 1 || exit 1; done
timeout -k 10 60 python tools/mb_probe.py C5_talos_walk 20 2048 || exit 1
timeout -k 10 60 python tools/mb_probe.py C4_solo12_trot 10 1 || exit 1
timeout -k 10 60 python tools/mb_probe.py C4_solo12_trot 10 4096 || exit 1
