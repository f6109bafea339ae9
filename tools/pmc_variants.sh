#!/bin/bash
# Two PMC passes (issue mix; F64 mix + memory) of one bench.py line per
# library variant: VARIANTS="base v1 ..." (base = the in-tree librtmi.so,
# else tools/ab/<v>.so), BENCH="bench.py args". Outputs under
# gpurun_out/$OUT/pmcv_<v>/{a,b}; summarise with tools/pmc_summary.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-pmcv}
K='k_render|k_frame_'
for v in ${VARIANTS:-base}; do
  P=$O/pmcv_$v
  mkdir -p $P
  if [ "$v" = base ]; then unset RTMI_LIB; else export RTMI_LIB=tools/ab/$v.so; fi
  timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES \
      --kernel-include-regex "$K" -d $P/a -o p -f csv -- python3 bench.py $BENCH > /dev/null 2> $P/a.err \
    && timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_BUSY_CYCLES \
      --kernel-include-regex "$K" -d $P/b -o p -f csv -- python3 bench.py $BENCH > /dev/null 2> $P/b.err \
    || { echo "pmc $v failed"; tail -5 $P/*.err; exit 1; }
  echo "pmc $v done"
done
