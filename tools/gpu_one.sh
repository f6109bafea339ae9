set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_bins.py > gpurun_out/one_tests.log 2>&1 || { tail -30 gpurun_out/one_tests.log; exit 1; }
tail -3 gpurun_out/one_tests.log
L=$(ls $PWD/tools/ab/*.so | tr "\n" "," | sed "s/,$//")
RTMI_LIBS=$L ABLATE=c3_full REPS=8 timeout -k 10 300 python tools/ab.py 2>&1 | grep -v stats | grep -v amdgpu.ids
