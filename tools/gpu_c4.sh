# C3 kernel split: general (k_render_gen1) vs lean (k_render_lean1q) pixels, serial launches
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c4
RTMI_SPLIT_SERIAL=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c4/trace -o run -f csv -- python bench.py --flags 1024 --steps 5 --warmup 2 --no-cpu > gpurun_out/c4/bench.log 2>&1 || exit 1
