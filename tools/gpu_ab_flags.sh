# interleaved A/B of tools/ab/*.so (FLAGSETS, CONFIG, REPS from the env), no tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
RTMI_LIBS=$(ls $PWD/tools/ab/*.so | tr '\n' ',' | sed 's/,$//') FLAGSETS=${FLAGSETS:-0} REPS=${REPS:-8} timeout -k 10 300 python -u tools/ab_flags.py > gpurun_out/ab_flags.log 2>&1
rc=$?; cat gpurun_out/ab_flags.log; exit $rc
