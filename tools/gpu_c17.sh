set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_queue.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c17_tests.log 2>&1 || { tail -30 gpurun_out/c17_tests.log; exit 1; }
tail -1 gpurun_out/c17_tests.log
