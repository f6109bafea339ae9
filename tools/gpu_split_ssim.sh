set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 200 --timeout-method thread > gpurun_out/split_tests.log 2>&1
rc=$?; tail -4 gpurun_out/split_tests.log; [ $rc -eq 0 ] || exit $rc
BANDS=4 timeout -k 10 300 python tools/scaling_sim.py > gpurun_out/ssim.json 2>gpurun_out/ssim.err; rc=$?; cat gpurun_out/ssim.json; exit $rc
