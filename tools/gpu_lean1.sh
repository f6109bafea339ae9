# split/parity/bins GPU tests, then C3 timing A/B (env var toggles)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/lean1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_bins.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -5 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  REPS=7 timeout -k 10 120 python tools/time_c3.py >> $O/time.json 2>>$O/time.err || exit 1
  RTMI_LEAN1Q=0 REPS=7 timeout -k 10 120 python tools/time_c3.py >> $O/time.json 2>>$O/time.err || exit 1
done
cat $O/time.json
