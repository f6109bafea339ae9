# Longest-first launch order: parity, per-launch overhead, scaling projection, bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests -m gpu -x -q > gpurun_out/gt.log 2>&1 && tail -1 gpurun_out/gt.log && \
CASES=bunny:16 timeout -k 10 300 python tools/tail_probe.py > gpurun_out/tail.log 2>&1 && \
BANDS=4 timeout -k 10 300 python tools/scaling_sim.py > gpurun_out/ss.json && \
timeout -k 10 600 python bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
echo rc=$?
tail -3 gpurun_out/gt.log; cat gpurun_out/tail.log gpurun_out/ss.json; cut -c1-200 gpurun_out/bench_c3.json
