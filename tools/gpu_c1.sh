# round-3 A/B: compaction tests + k_render_fast occupancy variants (tools/ab/*.so)
set -o pipefail
mkdir -p gpurun_out/c1
timeout -k 10 500 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_compact.py tests/test_gpu_frame.py > gpurun_out/c1/compact_tests.log 2>&1; rc=$?
echo "tests rc=$rc"
[ $rc -le 1 ] || exit $rc
for v in default wpe6 wpe5 wpe4 batch5; do
  if [ $v = default ]; then L=""; else L="$PWD/tools/ab/$v.so"; fi
  RTMI_LIB=$L timeout -k 10 200 python tools/scene_times.py boxes2:1920x1080:8 spheres-warm-3:512x512:1 spheres-reflection:1920x1080:8 mesh-mix:1920x1080:8 spheres-pointlight1:1920x1080:8 two-meshes:1920x1080:8 > gpurun_out/c1/ab_$v.log 2>&1 || exit 1
done
