# Round 4: per-call builds on the build stream overlapping the previous
# call's render (two buffer sets): the whole GPU suite, C3 / C2 bench lines
# with and without (RTMI_PIPE=0), the back-to-back scaling projection.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4i}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for pp in 1 0; do
  RTMI_PIPE=$pp timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > $O/c3_p$pp.json 2> $O/c3_p$pp.err || exit 1
  RTMI_PIPE=$pp timeout -k 10 200 python bench.py --config C2 --steps 20 --warmup 3 --no-cpu > $O/c2_p$pp.json 2> $O/c2_p$pp.err || exit 1
  echo pipe=$pp; cut -c1-260 $O/c3_p$pp.json; cut -c1-260 $O/c2_p$pp.json
done
REPS=20 BANDS=4 timeout -k 10 300 python tools/scaling_sim.py > $O/scaling_sim.json 2> $O/ss.err || exit 1
cat $O/scaling_sim.json
RTMI_PIPE=0 REPS=20 BANDS=4 timeout -k 10 300 python tools/scaling_sim.py > $O/scaling_sim_p0.json 2> $O/ss0.err || exit 1
cat $O/scaling_sim_p0.json
