# SAH bin count sweep: C3 and the 1M-face torus (C5 scene at 4K/256 spp)
cd $GRAFT_REPO_ROOT
for cfg in C3 C5; do for b in 32 8 16 64 128 32; do
  CONFIG=$cfg RTMI_SAH_BINS=$b timeout -k 10 200 python tools/time_c3.py || exit 1
done; done
