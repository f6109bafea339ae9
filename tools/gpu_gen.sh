# split/batched-kernel GPU tests, then the A/B of tools/ab/*.so x {default, NO_BATCH}
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/gen
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gen/tests.log 2>&1
rc=$?
tail -15 gpurun_out/gen/tests.log
[ $rc -eq 0 ] || exit $rc
RTMI_LIBS=$(ls $PWD/tools/ab/*.so | tr '\n' ',' | sed 's/,$//') FLAGSETS=0,0x20 REPS=${REPS:-6} timeout -k 10 300 python -u tools/ab_flags.py > gpurun_out/gen/ab.log 2>&1
rc=$?; cat gpurun_out/gen/ab.log; exit $rc
