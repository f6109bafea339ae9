# Round 4: atomic lists in k_frame_build2 for pipelined calls (RTMI_ALIST):
# tests, scaling projection with / without, rank-0 timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4z}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_pipe.py tests/test_gpu_split.py tests/test_gpu_dropin.py tests/test_gpu_multi.py tests/test_gpu_queue.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for al in 1 0 1 0; do
  RTMI_ALIST=$al REPS=20 BANDS=4 timeout -k 10 300 python tools/scaling_sim.py > $O/ss_$al.json 2> $O/ss_$al.err || exit 1
  echo "alist $al $(grep -o '"world8_b2b_max_ms": [0-9.]*' $O/ss_$al.json) $(grep -o '"world4_b2b_max_ms": [0-9.]*' $O/ss_$al.json) $(grep -o '"world2_b2b_max_ms": [0-9.]*' $O/ss_$al.json) $(grep -o '"world1_b2b_max_ms": [0-9.]*' $O/ss_$al.json) $(grep -o '"b2b_speedup_8": [0-9.]*' $O/ss_$al.json)"
done
REPS=30 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/t -o run -f csv -- python3 tools/rank_prof.py > $O/rp.log 2>&1 || exit 1
python3 tools/pipe_timeline.py $O/t/run_kernel_trace.csv
