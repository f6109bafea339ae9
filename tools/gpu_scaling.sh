set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/scal
timeout -k 10 300 python tools/scaling_sim.py > gpurun_out/scal/sim.jsonl 2> gpurun_out/scal/sim.err && \
timeout -k 10 300 python tools/host_overhead.py > gpurun_out/scal/loop.jsonl 2> gpurun_out/scal/loop.err && \
timeout -k 10 600 python bench.py > gpurun_out/scal/bench_c3.json 2> gpurun_out/scal/bench.err
rc=$?; cat gpurun_out/scal/sim.jsonl gpurun_out/scal/loop.jsonl; exit $rc
