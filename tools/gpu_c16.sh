set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_configs.py tests/test_gpu_frame.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c16_tests.log 2>&1 || { tail -30 gpurun_out/c16_tests.log; exit 1; }
tail -1 gpurun_out/c16_tests.log
VARIANTS="default scount" SCENES="mesh-bunny:1920x1080:16 mesh-bunny:3840x2160:32" REPS=3 bash tools/gpu_ab_scenes.sh
