# Diagnostics of the current build on C3: per-pixel-class cost map and the SQ
# instruction mix of the render kernel (one counter pass).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
K='k_render_fast<false'
RTMI_COST_DUMP=gpurun_out/diag/cost.bin timeout -k 10 200 python -u tools/cost_map.py > gpurun_out/diag/cost_map.json 2> gpurun_out/diag/cost_map.err && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "$K" -d gpurun_out/diag/pmc/sq -o p -f csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu > /dev/null 2> gpurun_out/diag/sq.err && \
python -c "import sys; sys.path.insert(0, 'tools'); import pmc_summary as m; m.main('gpurun_out/diag/pmc', 'diag_c3', out='gpurun_out/diag/pmc_summary.json')" > gpurun_out/diag/sq_summary.json
rc=$?
cat gpurun_out/diag/cost_map.json
echo rc=$rc
exit $rc
