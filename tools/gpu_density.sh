# C3 frame time vs light-grid density (RTMI_GRID_DENSITY, cells per listed face)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for dsty in ${DENS:-1 2 4 8 16}; do
  RTMI_GRID_DENSITY=$dsty REPS=9 timeout -k 10 120 python tools/time_c3.py || exit 1
done
