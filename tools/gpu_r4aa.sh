# Round 4: general-pixel batch size x occupancy on C3 (with LDS staging).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4aa}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -q --timeout 200 --timeout-method thread -k "c3" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in base b1 b1w8 b4w5; do
    L=""; [ $v != base ] && L=tools/ab/$v.so
    RTMI_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > $O/c3_${v}_$i.json 2> $O/c3_${v}_$i.err || exit 1
    echo "$v $i $(grep -o '"ms_per_step": [0-9.]*' $O/c3_${v}_$i.json) $(grep -o '"kernel_ms": [0-9.]*' $O/c3_${v}_$i.json)"
  done
done
