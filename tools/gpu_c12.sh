# C3 diagnostic: mesh-origin shadow rays' share (wrong images), serial two-kernel and merged
set -o pipefail
mkdir -p gpurun_out/c12
rm -rf gpurun_out/c12/*
for rep in 1 2; do
for v in default nomo; do
  if [ $v = default ]; then L=""; else L="$PWD/tools/ab/$v.so"; fi
  RTMI_SPLIT_SERIAL=1 RTMI_LIB=$L timeout -k 10 200 python tools/scene_times.py mesh-bunny+0x400:1920x1080:16 mesh-bunny:1920x1080:16 > gpurun_out/c12/ab_${v}_$rep.log 2>&1 || exit 1
done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_split.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c12/tests.log 2>&1 || { tail -20 gpurun_out/c12/tests.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c12/trace3 -o run -f csv -- python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/c12/bench3.log 2>&1 || exit 1
