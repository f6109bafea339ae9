set -o pipefail
mkdir -p gpurun_out/fuse
timeout -k 10 600 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_split.py tests/test_gpu_configs.py tests/test_gpu_bins.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fuse/tests.log 2>&1 || { tail -30 gpurun_out/fuse/tests.log; exit 1; }
tail -2 gpurun_out/fuse/tests.log
for r in 1 2; do
timeout -k 10 200 python tools/host_overhead.py > gpurun_out/fuse/ho_new_$r.json 2>/dev/null || exit 1
RTMI_LIB=$PWD/tools/ab/base.so timeout -k 10 200 python tools/host_overhead.py > gpurun_out/fuse/ho_base_$r.json 2>/dev/null || exit 1
done
head -20 gpurun_out/fuse/ho_*.json
VARIANTS="default base" SCENES="mesh-bunny:1920x1080:16 mesh-mix:1920x1080:8" REPS=3 bash tools/gpu_ab_scenes.sh && python tools/ab_report.py gpurun_out/ab setup_ms && python tools/ab_report.py gpurun_out/ab call_ms
