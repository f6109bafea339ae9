# Round 4: longer item runs per shard (each XCD takes every 8th stripe of a
# list: a smaller L2 footprint) on C3 and the N = 8 projection.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4cc}
mkdir -p $O
for i in 1 2; do
  for v in base g32 g128 g128l16 g512l64; do
    L=""; [ $v != base ] && L=tools/ab/$v.so
    RTMI_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > $O/c3_${v}_$i.json 2> $O/c3_${v}_$i.err || exit 1
    echo "$v $i $(grep -o '"ms_per_step": [0-9.]*' $O/c3_${v}_$i.json) $(grep -o '"kernel_ms": [0-9.]*' $O/c3_${v}_$i.json)"
  done
done
for v in base g128 g128l16 g512l64; do
  L=""; [ $v != base ] && L=tools/ab/$v.so
  RTMI_LIB=$L REPS=20 BANDS=4 timeout -k 10 300 python tools/scaling_sim.py > $O/ss_$v.json 2> $O/ss_$v.err || exit 1
  echo "$v $(grep -o '"world8_b2b_max_ms": [0-9.]*' $O/ss_$v.json) $(grep -o '"world4_b2b_max_ms": [0-9.]*' $O/ss_$v.json) $(grep -o '"world1_b2b_max_ms": [0-9.]*' $O/ss_$v.json)"
done
