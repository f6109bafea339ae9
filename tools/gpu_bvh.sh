# Device BVH builder: parity tests, then build/trace timing against the host SAH tree.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_bvh.py -m gpu -x -q > gpurun_out/bvh_t.log 2>&1
rc=$?
tail -30 gpurun_out/bvh_t.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/bvh_builders.py > gpurun_out/bvh_b.log 2>&1
rc=$?
cat gpurun_out/bvh_b.log
exit $rc
