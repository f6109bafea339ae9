# Round 4: pipelined builds by launch size (auto): pipe tests, the GPU suite,
# C3 bench, scaling projection, render time against launch size, LDS staging
# A/B (C3 x3 alternating, C5).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4j}
mkdir -p $O
#timeout -k 10 200 python -u -m pytest tests/test_gpu_pipe.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests_pipe.log 2>&1 || { tail -40 $O/tests_pipe.log; exit 1; }
#tail -2 $O/tests_pipe.log
#timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
#tail -2 $O/tests.log
#REPS=20 BANDS=4 timeout -k 10 300 python tools/scaling_sim.py > $O/scaling_sim.json 2> $O/ss.err || exit 1
#cat $O/scaling_sim.json
timeout -k 10 300 python tools/render_curve.py > $O/render_curve.jsonl 2> $O/rc.err || exit 1
cat $O/render_curve.jsonl
for i in 1 2 3; do
  for v in base lds; do
    L=""; [ $v = lds ] && L=tools/ab/lds.so
    RTMI_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > $O/c3_${v}_$i.json 2> $O/c3_${v}_$i.err || exit 1
    echo "$v $i $(cut -c1-190 $O/c3_${v}_$i.json | grep -o '"value": [0-9.]*, .*ms_per_step": [0-9.]*')"
  done
done
RTMI_LIB=tools/ab/lds.so timeout -k 10 300 python bench.py --config C5 --steps 3 --warmup 1 --no-cpu > $O/c5_lds.json 2> $O/c5_lds.err || exit 1
timeout -k 10 300 python bench.py --config C5 --steps 3 --warmup 1 --no-cpu > $O/c5_base.json 2> $O/c5_base.err || exit 1
cut -c1-200 $O/c5_lds.json; cut -c1-200 $O/c5_base.json
# C2 diagnostics (wrong images): the camera objects' / shadow objects' /
# normal pass's / all samples' share of the C2 render
for v in base nocam noshadow nonormal nosamples; do
  L=""; [ $v != base ] && L=tools/ab/$v.so
  RTMI_LIB=$L timeout -k 10 200 python bench.py --config C2 --steps 20 --warmup 3 --no-cpu > $O/c2_$v.json 2> $O/c2_$v.err || exit 1
  echo "c2 $v $(grep -o '"kernel_ms": [0-9.]*' $O/c2_$v.json)"
done
