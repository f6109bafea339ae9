set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/x16_tests.log 2>&1
rc=$?; tail -3 gpurun_out/x16_tests.log; [ $rc -eq 0 ] || exit $rc
RTMI_LIBS=$(ls $PWD/tools/ab/*.so | tr "\n" "," | sed "s/,$//") ABLATE=c3_full,boxes2_c2,bunny_only REPS=6 timeout -k 10 300 python tools/ab.py > gpurun_out/ab.log 2>&1; cat gpurun_out/ab.log | grep -v stats
