set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_bins.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sl_tests.log 2>&1
rc=$?; tail -3 gpurun_out/sl_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
REPS=7 timeout -k 10 120 python tools/time_c3.py | cut -c1-100 || exit 1
RTMI_NO_SHADOW_LISTS=1 REPS=7 timeout -k 10 120 python tools/time_c3.py | cut -c1-100 || exit 1
done
