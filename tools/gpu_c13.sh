set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_bins.py tests/test_gpu_configs.py::test_c2_1080p_64spp_rows tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c13_tests.log 2>&1 || { tail -20 gpurun_out/c13_tests.log; exit 1; }
tail -1 gpurun_out/c13_tests.log
VARIANTS="default" SCENES="boxes2:1920x1080:8 spheres-warm:1920x1080:8 spheres-pointlight1:1920x1080:8" REPS=2 bash tools/gpu_ab_scenes.sh
