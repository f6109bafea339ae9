cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
RTMI_LIBS=$PWD/tools/ab/t0.so,$PWD/tools/ab/t1v.so timeout -k 10 300 python -u tools/order_check.py > gpurun_out/order_check.json 2> gpurun_out/order_check.err
