# Round 4: LDS staging by default + pipelined small launches: the GPU suite,
# C3 bench, no-LDS A/B, scaling projection.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4m}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for v in base nolds; do
    L=""; [ $v != base ] && L=tools/ab/$v.so
    RTMI_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > $O/c3_${v}_$i.json 2> $O/c3_${v}_$i.err || exit 1
    echo "$v $i $(grep -o '"ms_per_step": [0-9.]*' $O/c3_${v}_$i.json) $(grep -o '"kernel_ms": [0-9.]*' $O/c3_${v}_$i.json)"
  done
done
REPS=20 BANDS=4 timeout -k 10 300 python tools/scaling_sim.py > $O/scaling_sim.json 2> $O/ss.err || exit 1
cat $O/scaling_sim.json
