# Round 4: XCD-chunked work queues (RTMI_XCD_CHUNK) x LDS staging A/B on C3,
# scaling projection and C5; parity tests of the mix kernel first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4l}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipe.py tests/test_gpu_split.py tests/test_gpu_configs.py tests/test_gpu_frame.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for v in base nochunk lds ldschunk0; do
    L=""; [ $v != base ] && L=tools/ab/$v.so
    RTMI_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > $O/c3_${v}_$i.json 2> $O/c3_${v}_$i.err || exit 1
    echo "$v $i $(grep -o '"ms_per_step": [0-9.]*' $O/c3_${v}_$i.json) $(grep -o '"kernel_ms": [0-9.]*' $O/c3_${v}_$i.json)"
  done
done
for v in base nochunk; do
  L=""; [ $v != base ] && L=tools/ab/$v.so
  RTMI_LIB=$L REPS=20 BANDS=4 timeout -k 10 300 python tools/scaling_sim.py > $O/ss_$v.json 2> $O/ss_$v.err || exit 1
  echo $v; cat $O/ss_$v.json
  RTMI_LIB=$L timeout -k 10 300 python bench.py --config C5 --steps 3 --warmup 1 --no-cpu > $O/c5_$v.json 2> $O/c5_$v.err || exit 1
  echo "c5 $v $(grep -o '"ms_per_step": [0-9.]*' $O/c5_$v.json)"
done
