# Parity suite + one bench line per BASELINE config on one GPU.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests -m gpu -x -q > gpurun_out/gt.log 2>&1; tail -1 gpurun_out/gt.log
timeout -k 10 600 python bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err && \
timeout -k 10 300 python bench.py --config C2 --no-cpu > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err && \
timeout -k 10 600 python bench.py --config C4 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err && \
timeout -k 10 900 python bench.py --config C5 --steps 2 --warmup 1 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err
echo rc=$?
