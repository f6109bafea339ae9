# round-3 A/B of the big-face threshold (setup time), + frame-list tests on the extreme variant
set -o pipefail
mkdir -p gpurun_out/c3
rm -f gpurun_out/c3/*.log
RTMI_LIB=$PWD/tools/ab/big16.so timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_frame.py > gpurun_out/c3/tests_big16.log 2>&1 || exit 1
for rep in 1 2; do
for v in default big16 big128 big256 big1024 big100000; do
  if [ $v = default ]; then L=""; else L="$PWD/tools/ab/$v.so"; fi
  RTMI_LIB=$L timeout -k 10 200 python tools/scene_times.py mesh-bunny:1920x1080:16 mesh-mix:1920x1080:8 mesh-bunny:3840x2160:32 two-meshes:1920x1080:8 > gpurun_out/c3/ab_${v}_$rep.log 2>&1 || exit 1
done
done
