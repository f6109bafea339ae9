# PMC passes (one counter group per rocprofv3 run, no tracing domains) of the
# bench command for each BASELINE config: FETCH_SIZE, WRITE_SIZE, then the SQ
# issue counters. Summarise afterwards on the CPU with
#   python tools/pmc_summary.py gpurun_out/pmc_<cfg> <workload key> "<note>"
# CONFIGS="C3 C2 C4 C5" (default); each pass under its own time limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
K='k_render_fast<false|k_render_lean|k_render_gen|k_render_mix1|k_frame_'
for cfg in ${CONFIGS:-C3 C2 C4 C5}; do
  c=$(echo $cfg | tr A-Z a-z)
  O=gpurun_out/pmc_$c
  mkdir -p $O
  T=120; [ $cfg = C5 ] && T=400; [ $cfg = C4 ] && T=200
  timeout -s KILL $T rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $O/fetch -o p -f csv -- python3 bench.py --config $cfg --steps 2 --warmup 0 --no-cpu > /dev/null 2> $O/fetch.err || { echo "$cfg fetch failed"; tail -5 $O/fetch.err; exit 1; }
  timeout -s KILL $T rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $O/write -o p -f csv -- python3 bench.py --config $cfg --steps 2 --warmup 0 --no-cpu > /dev/null 2> $O/write.err || { echo "$cfg write failed"; exit 1; }
  timeout -s KILL $T rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "$K" -d $O/sq -o p -f csv -- python3 bench.py --config $cfg --steps 2 --warmup 0 --no-cpu > /dev/null 2> $O/sq.err || { echo "$cfg sq failed"; exit 1; }
  echo "$cfg pmc done"
done
