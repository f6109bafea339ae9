# Round 4: item runs per shard (framebuffer write-backs) x gen1 occupancy x
# LDS staging scope on C3: split tests, time A/B, WRITE_SIZE per variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4q}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_configs.py tests/test_gpu_pipe.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for v in base run1 w6 lds3 w6run1; do
    L=""; [ $v != base ] && L=tools/ab/$v.so
    RTMI_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > $O/c3_${v}_$i.json 2> $O/c3_${v}_$i.err || exit 1
    echo "$v $i $(grep -o '"ms_per_step": [0-9.]*' $O/c3_${v}_$i.json) $(grep -o '"kernel_ms": [0-9.]*' $O/c3_${v}_$i.json)"
  done
done
for v in base run1 w6; do
  L=""; [ $v != base ] && L=tools/ab/$v.so
  RTMI_LIB=$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_render_mix1" -d $O/w_$v -o p -f csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu > /dev/null 2> $O/w_$v.err || exit 1
  python3 - <<PY
import csv
v=[float(r["Counter_Value"]) for r in csv.DictReader(open("$O/w_$v/p_counter_collection.csv")) if "mix1" in r["Kernel_Name"]]
print("$v WRITE_SIZE MB per dispatch", round(sum(v)/max(1,len(v)/1)*1024/1e6, 1) if False else [round(x*1024/1e6,1) for x in v][:6])
PY
done
