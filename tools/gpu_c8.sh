# GPU tests, then C3 / C4 timings (scene_times) and the kernel trace of the C3 bench
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c8
rm -rf gpurun_out/c8/*
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c8/tests.log 2>&1 || { tail -30 gpurun_out/c8/tests.log; exit 1; }
tail -2 gpurun_out/c8/tests.log
timeout -k 10 200 python tools/scene_times.py mesh-bunny:1920x1080:16 mesh-bunny:3840x2160:32 mesh-mix:1920x1080:8 boxes2:1920x1080:8 > gpurun_out/c8/times.log 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c8/trace -o run -f csv -- python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/c8/bench.log 2>&1 || exit 1
