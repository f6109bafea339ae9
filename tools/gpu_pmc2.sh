cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in ground_nolights c3_full; do
ABLATE=$v timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_SALU SQ_INSTS_VALU --kernel-include-regex "k_render<float, false>" -d gpurun_out/pmc2/$v/a -o p -f csv -- python3 tools/ablate.py > /dev/null 2>&1 || exit 1
ABLATE=$v timeout -k 10 200 rocprofv3 --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SMEM SQ_INSTS_VMEM_RD --kernel-include-regex "k_render<float, false>" -d gpurun_out/pmc2/$v/b -o p -f csv -- python3 tools/ablate.py > /dev/null 2>&1 || exit 1
done
