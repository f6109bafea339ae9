set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
export OUT=${OUT:-r6fb}
STAGES="pmc:C3 pmc:C3:fp64 pmc:C3:bvh pmc:C2 pmc:BVHMIX" bash tools/gpu_job.sh || exit 1
O=gpurun_out/$OUT; K='k_render|k_frame_'
# typed VALU mix of the C3 render kernels (the spill-share bound)
P=$O/pmc_c3_typed; mkdir -p $P
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 \
  --kernel-include-regex "$K" -d $P/typed -o p -f csv -- python3 bench.py --config C3 --steps 2 --warmup 0 --no-cpu --no-extra > /dev/null 2> $P/typed.err || { tail -5 $P/typed.err; exit 1; }
echo finalB ok
