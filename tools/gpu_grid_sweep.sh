# GPU tests, then the A/B of tools/ab/*.so, then light-grid density sweep of the in-tree build
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
RTMI_LIBS=$(ls $PWD/tools/ab/*.so | tr '\n' ',' | sed 's/,$//') ABLATE=c3_full,c3_nolights,ground_only timeout -k 10 300 python -u tools/ab.py > gpurun_out/ab.log 2>&1 && \
for dd in 2 4 8 16; do RTMI_GRID_DENSITY=$dd RTMI_LIBS=$PWD/nim-raytracer_amd/rtmi/librtmi.so ABLATE=c3_full REPS=3 timeout -k 10 120 python -u tools/ab.py > gpurun_out/grid_$dd.log 2>&1 || exit 1; done
