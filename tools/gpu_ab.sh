cd $GRAFT_REPO_ROOT
libs=$(ls $PWD/tools/ab/*.so | tr '\n' ',' | sed 's/,$//')
RTMI_LIBS=$libs timeout -k 10 600 python tools/ab.py > gpurun_out/ab.log 2>&1
