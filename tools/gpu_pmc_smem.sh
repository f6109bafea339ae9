# Scalar-cache and scalar-load latency counters of the C3 render kernel (one pass per group).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
K='k_render_fast<false'
R() { REPS=1 timeout -k 10 200 rocprofv3 --pmc "$@" --kernel-include-regex "$K" -d gpurun_out/pmcs/$1 -o p -f csv -- python3 tools/time_c3.py > /dev/null 2> gpurun_out/pmcs_$1.err || exit 1; }
R SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE
R SQ_INST_LEVEL_SMEM SQ_ACCUM_PREV_HIRES SQ_INSTS_SMEM
R SQ_WAIT_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SMEM SQ_WAVE_CYCLES SQ_INSTS_SALU
R SQC_TC_DATA_READ_REQ SQC_TC_STALL SQC_DCACHE_BUSY_CYCLES SQ_BUSY_CU_CYCLES
