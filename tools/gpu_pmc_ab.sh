cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for lib in tools/ab/*.so; do
  n=$(basename $lib .so)
  RTMI_LIBS=$PWD/$lib REPS=1 ABLATE=${ABLATE:-c3_full} timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex "k_render_fast<false>" -d gpurun_out/pmcab/$n -o p -f csv -- python3 tools/ab.py > gpurun_out/pmcab_$n.log 2>&1 || exit 1
done
