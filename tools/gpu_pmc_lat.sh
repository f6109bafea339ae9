# Latency / cache PMC passes of the render kernel on one ablation variant (default c3_full)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
LIB=${LIB:-$PWD/nim-raytracer_amd/rtmi/librtmi.so}
V=${V:-c3_full}
run() { RTMI_LIBS=$LIB REPS=1 ABLATE=$V timeout -s KILL 120 rocprofv3 --pmc $2 --kernel-include-regex "k_render_fast<false" -d gpurun_out/pmclat/$V/$1 -o p -f csv -- python3 tools/ab.py > gpurun_out/pmclat_$1.log 2>&1; }
run a "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_MISSES_DUPLICATE SQC_DCACHE_REQ SQC_TC_DATA_READ_REQ SQC_TC_STALL SQC_ICACHE_HITS SQC_ICACHE_MISSES" && \
run b "SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_SALU" && \
run c "TCC_HIT_sum TCC_MISS_sum" && \
run d "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_IFETCH SQ_CYCLES" && \
python3 tools/pmc_show.py gpurun_out/pmclat/$V > gpurun_out/pmclat_$V.txt
