cd $GRAFT_REPO_ROOT
export ABLATE=c3_full,ground_nolights,bunny_only
for w in 4 5 6 8; do
  RTMI_LIB=$PWD/tools/librtmi_w$w.so TAG=_w$w timeout -k 10 200 python tools/ablate.py > gpurun_out/occ_w$w.log 2>&1 || exit 1
done
