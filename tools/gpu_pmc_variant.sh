# SQ instruction mix of the render kernel on tools/ab.py variants (current
# build only): VARIANTS="lean_only c3_full" bash tools/gpu_pmc_variant.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcv
K=${K:-'k_render_fast<false'}
for v in ${VARIANTS:-lean_only c3_full}; do
  RTMI_LIBS=$PWD/nim-raytracer_amd/rtmi/librtmi.so ABLATE=$v REPS=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "$K" -d gpurun_out/pmcv/$v/sq -o p -f csv -- python3 tools/ab.py > gpurun_out/pmcv/$v.log 2>&1 || exit 1
  python -c "import sys; sys.path.insert(0, 'tools'); import pmc_summary as m; m.KERNEL = \"$K\"; m.main('gpurun_out/pmcv/$v', '$v', out='gpurun_out/pmcv/summary.json')" > /dev/null || exit 1
done
python - <<'PY'
import json
d = json.load(open("gpurun_out/pmcv/summary.json"))
for k, e in d.items():
    c = e["counters_mean_per_dispatch"]
    print(k, {n: f"{v:.4g}" for n, v in sorted(c.items())})
PY
