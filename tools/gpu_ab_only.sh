# interleaved A/B of tools/ab/*.so (no tests)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
RTMI_LIBS=$(ls $PWD/tools/ab/*.so | tr '\n' ',' | sed 's/,$//') ABLATE=${ABLATE:-c3_full,c3_nolights} REPS=${REPS:-8} timeout -k 10 600 python -u tools/ab.py > gpurun_out/ab.log 2>&1
