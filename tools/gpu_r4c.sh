# Round 4: the two-launch build + spill-free one-plane kernels. Build tests,
# the whole GPU suite, the C3 bench line, a kernel trace, then A/B against the
# round-3 library (tools/ab/r3.so) and the two-virtual-lane lean loop
# (tools/ab/h2.so), and the multi-GPU projection (rank-0 loop + every rank).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4c}
mkdir -p $O
export RTMI_PARITY_LOG=$PWD/$O/parity.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_dropin.py tests/test_gpu_split.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests_build.log 2>&1 || { tail -40 $O/tests_build.log; exit 1; }
tail -2 $O/tests_build.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --deselect tests/test_gpu_frame.py --deselect tests/test_gpu_dropin.py --deselect tests/test_gpu_split.py > $O/tests_all.log 2>&1 || { tail -40 $O/tests_all.log; exit 1; }
tail -2 $O/tests_all.log
timeout -k 10 300 python bench.py --no-cpu > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
cut -c1-400 $O/bench_c3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $O/bench_prof.json 2> $O/prof.err || exit 1
timeout -k 10 300 python tools/host_overhead.py > $O/host_overhead.json 2> $O/ho.err || exit 1
cat $O/host_overhead.json
BANDS=4 timeout -k 10 300 python tools/scaling_sim.py > $O/scaling_sim.json 2> $O/ss.err || exit 1
cat $O/scaling_sim.json
VARIANTS="default r3 h2 hitf" SCENES="mesh-bunny:1920x1080:16 mesh-mix:1920x1080:8 boxes2:1920x1080:8" REPS=3 bash tools/gpu_ab_scenes.sh || exit 1
mkdir -p $O/ab && cp gpurun_out/ab/*.log $O/ab/
python tools/ab_report.py gpurun_out/ab setup_ms; python tools/ab_report.py gpurun_out/ab call_ms
RTMI_LIB=$PWD/tools/ab/lanes.so RTMI_STAT_FLUSH=1 timeout -k 10 300 python tools/lanes_probe.py > $O/lanes_probe.json 2> $O/lanes.err || exit 1
cat $O/lanes_probe.json
# row n1 on C5 (the scene that overflows L2): LDS-staged face records A/B
VARIANTS="default lds" SCENES="torus:3840x2160:64" REPS=2 bash tools/gpu_ab_scenes.sh || exit 1
mkdir -p $O/ab_lds && cp gpurun_out/ab/*.log $O/ab_lds/
python tools/ab_report.py gpurun_out/ab render_ms
# C2 (boxes2) cost breakdown: diagnostic builds with parts of the object-binned batch switched off (wrong images, timing only)
VARIANTS="default hitf obnoshadow obnocam obnonormal nosamples" SCENES="boxes2:1920x1080:8" REPS=2 bash tools/gpu_ab_scenes.sh || exit 1
mkdir -p $O/ab_c2 && cp gpurun_out/ab/*.log $O/ab_c2/
python tools/ab_report.py gpurun_out/ab render_ms
