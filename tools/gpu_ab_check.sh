# GPU tests, A/B of tools/ab/head.so vs the other build, and the fp32-vs-fp64 hit check
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
RTMI_LIBS=$(ls $PWD/tools/ab/*.so | tr '\n' ',' | sed 's/,$//') ABLATE=${ABLATE:-c3_full,c3_nolights,ground_only,boxes2_c2} REPS=${REPS:-4} timeout -k 10 300 python -u tools/ab.py > gpurun_out/ab.log 2>&1 && \
RTMI_LIBS=$(ls $PWD/tools/ab/*.so | tr '\n' ',' | sed 's/,$//') timeout -k 10 300 python -u tools/order_check.py > gpurun_out/order_check.json 2> gpurun_out/order_check.err
