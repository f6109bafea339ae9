# Round 4, first GPU call: the new drop-in / overflow / full-frame tests first,
# then the whole GPU suite, then the C3 bench line (fp32) and the fp64
# parity-mode line. Each step under its own time limit, chained with &&.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
export RTMI_PARITY_LOG=$PWD/$O/parity.jsonl
timeout -k 10 400 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests_new.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread --deselect tests/test_gpu_configs.py --deselect tests/test_gpu_dropin.py > $O/tests_all.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err && \
timeout -k 10 300 python bench.py --precision fp64 --steps 3 --warmup 1 --no-cpu > $O/bench_c3_fp64.json 2> $O/bench_c3_fp64.err
rc=$?
tail -3 $O/tests_new.log $O/tests_all.log
cat $O/bench_c3.json $O/bench_c3_fp64.json 2>/dev/null | cut -c1-400
exit $rc
