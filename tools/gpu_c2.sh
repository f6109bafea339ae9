# round-3 occupancy A/B, interleaved repetitions (tools/ab/*.so)
set -o pipefail
mkdir -p gpurun_out/c2
rm -f gpurun_out/c2/*.log
for rep in 1 2 3; do
for v in default m6 m7 perray lds; do
  if [ $v = default ]; then L=""; else L="$PWD/tools/ab/$v.so"; fi
  RTMI_LIB=$L timeout -k 10 200 python tools/scene_times.py boxes2:1920x1080:8 mesh-mix:1920x1080:8 two-meshes:1920x1080:8 mesh-bunny:1920x1080:2 mesh-bunny+0x10:1920x1080:16 mesh-bunny:1920x1080:16 spheres-warm-3:512x512:1 > gpurun_out/c2/ab_${v}_$rep.log 2>&1 || exit 1
done
done
