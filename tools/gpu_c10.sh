# C2 kernel trace (per-call build kernels)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c10
rm -rf gpurun_out/c10/*
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c10/trace -o run -f csv -- python bench.py --config C2 --steps 5 --warmup 2 --no-cpu > gpurun_out/c10/bench.log 2>&1 || exit 1
