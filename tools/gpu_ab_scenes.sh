# A/B of library builds (tools/build_variant.sh -> tools/ab/NAME.so; "default"
# = the in-tree librtmi.so) on scene timings (tools/scene_times.py), the
# variants interleaved over REPS repetitions; logs in gpurun_out/ab/ (summarise
# with tools/ab_report.py). Extra environment (e.g. RTMI_SPLIT_SERIAL=1) passes
# through.
#   VARIANTS="default nocut" SCENES="mesh-bunny:1920x1080:16" REPS=2 bash tools/gpu_ab_scenes.sh
set -o pipefail
mkdir -p gpurun_out/ab
rm -f gpurun_out/ab/*.log
for rep in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-default}; do
    if [ "$v" = default ]; then L=""; else L="$PWD/tools/ab/$v.so"; fi
    RTMI_LIB=$L timeout -k 10 300 python tools/scene_times.py ${SCENES:-mesh-bunny:1920x1080:16} > gpurun_out/ab/ab_${v}_$rep.log 2>&1 || exit 1
  done
done
