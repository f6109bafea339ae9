# Round 4: lean items of 16 pixels down to one item per resident wave:
# tests, scaling projection, rank-0 timeline at N = 8, shard caps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4u}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_pipe.py tests/test_gpu_multi.py tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
REPS=20 BANDS=4 timeout -k 10 300 python tools/scaling_sim.py > $O/ss.json 2> $O/ss.err || exit 1
cat $O/ss.json
REPS=30 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/t -o run -f csv -- python3 tools/rank_prof.py > $O/rp.log 2>&1 || exit 1
python3 tools/pipe_timeline.py $O/t/run_kernel_trace.csv
for sh in 16 32; do
  RTMI_SHARDS=$sh REPS=20 BANDS=4 timeout -k 10 300 python tools/scaling_sim.py > $O/ss_sh$sh.json 2> $O/ss_sh$sh.err || exit 1
  echo "shards $sh $(grep -o '"world8_b2b_max_ms": [0-9.]*' $O/ss_sh$sh.json) $(grep -o '"world1_b2b_max_ms": [0-9.]*' $O/ss_sh$sh.json)"
done
