# One GPU call: smoke, GPU parity tests, the default bench line, rocprofv3 kernel stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r1 -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_prof.json 2> gpurun_out/prof.err
