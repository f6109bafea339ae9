# GPU tests, then setup / render timings of the main scenes
set -o pipefail
mkdir -p gpurun_out/c9
rm -rf gpurun_out/c9/*
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c9/tests.log 2>&1 || { tail -30 gpurun_out/c9/tests.log; exit 1; }
tail -2 gpurun_out/c9/tests.log
timeout -k 10 200 python tools/scene_times.py mesh-bunny:1920x1080:16 boxes2:1920x1080:8 mesh-bunny:3840x2160:32 mesh-mix:1920x1080:8 > gpurun_out/c9/times.log 2>&1 || exit 1
