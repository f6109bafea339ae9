# Round 4: the two-launch per-call build (slot lists + look-back): the frame /
# drop-in / split tests first (they exercise the build), then the whole GPU
# suite, then the C3 bench line and a rocprofv3 kernel trace of it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4b}
mkdir -p $O
export RTMI_PARITY_LOG=$PWD/$O/parity.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_dropin.py tests/test_gpu_split.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests_build.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_frame.py --deselect tests/test_gpu_dropin.py --deselect tests/test_gpu_split.py > $O/tests_all.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu > $O/bench_c3.json 2> $O/bench_c3.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $O/bench_prof.json 2> $O/prof.err
rc=$?
tail -3 $O/tests_build.log; tail -3 $O/tests_all.log
cut -c1-300 $O/bench_c3.json 2>/dev/null
exit $rc
