set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/s3
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/s3/smoke.log 2>&1 && \
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/s3/tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/s3/bench.json 2> gpurun_out/s3/bench.err
rc=$?; tail -3 gpurun_out/s3/tests.log; cat gpurun_out/s3/bench.json; echo rc=$rc; exit $rc
