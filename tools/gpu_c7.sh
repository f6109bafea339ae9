# depth cut A/B (C3 and friends) after the GPU tests
set -o pipefail
mkdir -p gpurun_out/c7
rm -f gpurun_out/c7/*.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c7/tests.log 2>&1 || { tail -30 gpurun_out/c7/tests.log; exit 1; }
tail -2 gpurun_out/c7/tests.log
for rep in 1 2; do
for v in default nocut; do
  if [ $v = default ]; then L=""; else L="$PWD/tools/ab/$v.so"; fi
  RTMI_LIB=$L timeout -k 10 200 python tools/scene_times.py mesh-bunny:1920x1080:16 mesh-bunny:3840x2160:32 two-meshes:1920x1080:8 torus:1920x1080:8 > gpurun_out/c7/ab_${v}_$rep.log 2>&1 || exit 1
done
done
