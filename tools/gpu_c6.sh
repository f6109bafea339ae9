# C3 general-pixel kernel (k_render_gen1, standalone: NO_MIX + serial) with its parts switched off (diagnostic builds, wrong images)
set -o pipefail
mkdir -p gpurun_out/c6
rm -f gpurun_out/c6/*.log
for rep in 1 2; do
for v in default NOCAM NOSHADOW NOSHADOWSEARCH NOTESTS; do
  if [ $v = default ]; then L=""; else L="$PWD/tools/ab/$v.so"; fi
  RTMI_SPLIT_SERIAL=1 RTMI_LIB=$L timeout -k 10 200 python tools/scene_times.py mesh-bunny+0x400:1920x1080:16 > gpurun_out/c6/ab_${v}_$rep.log 2>&1 || exit 1
done
done
