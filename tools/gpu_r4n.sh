# Round 4: the pipelined rank-0 loop at N = 8: kernel-trace timelines with
# the default build stream, a high-priority one, and capped render grids.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4n}
mkdir -p $O
for v in "def" "prio RTMI_PIPE_PRIO=1" "g90 RTMI_PIPE_GRID=90" "g80 RTMI_PIPE_GRID=80" "nopipe RTMI_PIPE=0"; do
  set -- $v
  env $2 REPS=30 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/t_$1 -o run -f csv -- python3 tools/rank_prof.py > $O/rp_$1.log 2>&1 || exit 1
  echo "$1 $(python3 tools/pipe_timeline.py $O/t_$1/run_kernel_trace.csv)"
done
for v in "prio RTMI_PIPE_PRIO=1" "g90 RTMI_PIPE_GRID=90"; do
  set -- $v
  env $2 REPS=20 BANDS=4 timeout -k 10 300 python tools/scaling_sim.py > $O/ss_$1.json 2> $O/ss_$1.err || exit 1
  echo "$1 $(cat $O/ss_$1.json)"
done
