# Round 4: event release scope (RTMI_EVENT_SCOPE 0 / 1 / 2) against the
# pipelined rank loop and the whole-frame bench; pipe tests first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4v}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_multi.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for sc in 1 0 2; do
  RTMI_EVENT_SCOPE=$sc REPS=20 BANDS=4 timeout -k 10 300 python tools/scaling_sim.py > $O/ss_$sc.json 2> $O/ss_$sc.err || exit 1
  RTMI_EVENT_SCOPE=$sc timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > $O/c3_$sc.json 2> $O/c3_$sc.err || exit 1
  echo "scope $sc $(grep -o '"world8_b2b_max_ms": [0-9.]*' $O/ss_$sc.json) $(grep -o '"world4_b2b_max_ms": [0-9.]*' $O/ss_$sc.json) $(grep -o '"world1_b2b_max_ms": [0-9.]*' $O/ss_$sc.json) c3 $(grep -o '"ms_per_step": [0-9.]*' $O/c3_$sc.json)"
done
