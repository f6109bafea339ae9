# C3 A/B: light-grid density (RTMI_GRID_DENSITY) and gen1/mix1 occupancy variants
set -o pipefail
mkdir -p gpurun_out/c5
rm -f gpurun_out/c5/*.log
for rep in 1 2; do
for dens in 1 2 4 8; do
  RTMI_GRID_DENSITY=$dens timeout -k 10 200 python tools/scene_times.py mesh-bunny:1920x1080:16 mesh-bunny+0x400:1920x1080:16 > gpurun_out/c5/ab_d${dens}_$rep.log 2>&1 || exit 1
done
for v in g6 g8; do
  RTMI_LIB=$PWD/tools/ab/$v.so timeout -k 10 200 python tools/scene_times.py mesh-bunny:1920x1080:16 mesh-bunny+0x400:1920x1080:16 > gpurun_out/c5/ab_${v}_$rep.log 2>&1 || exit 1
done
done
