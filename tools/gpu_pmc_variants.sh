# PMC instruction counters of the render kernel per ablation variant (tools/ab.py ABLATE names)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
LIB=${LIB:-$PWD/nim-raytracer_amd/rtmi/librtmi.so}
for v in ${VARIANTS:-ground_nolights ground_only bunny_only c3_nolights c3_full boxes2_c2}; do
  RTMI_LIBS=$LIB REPS=1 ABLATE=$v timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex "k_render_fast<false" -d gpurun_out/pmcvar/$v -o p -f csv -- python3 tools/ab.py > gpurun_out/pmcvar_$v.log 2>&1 || exit 1
done
