# GPU parity tests of the in-tree build, then an interleaved A/B of tools/ab/*.so
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
RTMI_LIBS=$(ls $PWD/tools/ab/*.so | tr '\n' ',' | sed 's/,$//') ABLATE=${ABLATE:-c3_full,c3_nolights,ground_only,boxes2_c2} timeout -k 10 600 python -u tools/ab.py > gpurun_out/ab.log 2>&1
