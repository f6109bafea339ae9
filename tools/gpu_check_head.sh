# Quick state check of HEAD on one MI355X: smoke, GPU tests, C3 bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/head
mkdir -p $O
timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err
rc=$?
tail -3 $O/tests.log
cat $O/bench_c3.json
echo rc=$rc
exit $rc
