cd $GRAFT_REPO_ROOT
timeout -k 10 500 python tools/ablate.py > gpurun_out/ablate.log 2>&1
