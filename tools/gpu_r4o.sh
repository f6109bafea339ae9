# Round 4: three rotating buffer sets, one event per call: pipe tests, the
# rank-0 timelines at N = 8, scaling projection, C3 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4o}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_dropin.py tests/test_gpu_multi.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for v in "def" "prio RTMI_PIPE_PRIO=1" "nopipe RTMI_PIPE=0"; do
  set -- $v
  env $2 REPS=30 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/t_$1 -o run -f csv -- python3 tools/rank_prof.py > $O/rp_$1.log 2>&1 || exit 1
  echo "$1 $(python3 tools/pipe_timeline.py $O/t_$1/run_kernel_trace.csv)"
done
for v in "def" "prio RTMI_PIPE_PRIO=1"; do
  set -- $v
  env $2 REPS=20 BANDS=4 timeout -k 10 300 python tools/scaling_sim.py > $O/ss_$1.json 2> $O/ss_$1.err || exit 1
  echo "$1 $(cat $O/ss_$1.json)"
done
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > $O/c3.json 2> $O/c3.err || exit 1
echo "c3 $(grep -o '"ms_per_step": [0-9.]*' $O/c3.json) $(grep -o '"kernel_ms": [0-9.]*' $O/c3.json)"
