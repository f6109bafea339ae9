# GPU tests, scene timings, C2 + C3 kernel traces
set -o pipefail
bash tools/gpu_c9.sh || exit 1
bash tools/gpu_c10.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c10/trace3 -o run -f csv -- python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/c10/bench3.log 2>&1 || exit 1
