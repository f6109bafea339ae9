# Round 4: compacted light-cell searches in gen1 (RTMI_GEN1_COMPACT) A/B,
# its occupancy variant, longer item runs; parity tests first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4r}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for v in base nocmp cmpw6 run16; do
    L=""; [ $v != base ] && L=tools/ab/$v.so
    RTMI_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > $O/c3_${v}_$i.json 2> $O/c3_${v}_$i.err || exit 1
    echo "$v $i $(grep -o '"ms_per_step": [0-9.]*' $O/c3_${v}_$i.json) $(grep -o '"kernel_ms": [0-9.]*' $O/c3_${v}_$i.json)"
  done
done
for v in base nocmp; do
  L=""; [ $v != base ] && L=tools/ab/$v.so
  RTMI_LIB=$L timeout -k 10 300 python bench.py --config C5 --steps 3 --warmup 1 --no-cpu > $O/c5_$v.json 2> $O/c5_$v.err || exit 1
  echo "c5 $v $(grep -o '"ms_per_step": [0-9.]*' $O/c5_$v.json)"
done
