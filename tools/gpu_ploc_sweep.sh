set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for r in 16 8 32; do
  echo "radius=$r"
  RTMI_PLOC_RADIUS=$r timeout -k 10 300 python tools/bvh_builders.py 2>&1 | grep ploc || exit 1
done
