# Round 4: C2 object-binned batches walking the samples' light cells jointly
# (RTMI_OB_CELLS_JOINT) A/B; the tests that cover boxes2 first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4s}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bins.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2 3; do
  for v in base cellsk; do
    L=""; [ $v != base ] && L=tools/ab/$v.so
    RTMI_LIB=$L timeout -k 10 200 python bench.py --config C2 --steps 30 --warmup 3 --no-cpu > $O/c2_${v}_$i.json 2> $O/c2_${v}_$i.err || exit 1
    echo "$v $i $(grep -o '"ms_per_step": [0-9.]*' $O/c2_${v}_$i.json) $(grep -o '"kernel_ms": [0-9.]*' $O/c2_${v}_$i.json)"
  done
done
