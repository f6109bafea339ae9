cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 300 python -u tools/ablate.py > gpurun_out/ablate.log 2>&1 && \
RTMI_LIB=tools/ab/stamps1.so ABLATE=c3_full,ground_nolights,c3_nolights timeout -k 10 200 python -u tools/stamps.py > gpurun_out/stamps1.log 2>&1 && \
RTMI_LIB=tools/ab/stamps2.so ABLATE=c3_full timeout -k 10 200 python -u tools/stamps.py > gpurun_out/stamps2.log 2>&1
