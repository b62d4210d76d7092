set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r05po}
mkdir -p $O
timeout -k 10 60 python tools/mb_probe.py C5_talos_walk ${KNOT:-20} ${NWG:-2048} > $O/probe_tree.log 2>&1 || { tail $O/probe_tree.log; exit 1; }
