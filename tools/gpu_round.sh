# One GPU call: GPU tests, then bench lines and rocprofv3 passes of the C3
# bench. STAGES picks the parts (default "tests bench prof"); outputs under
# gpurun_out/round/ (copied into profiles/ afterwards). Every GPU step has its
# own time limit and the steps are chained with && (nothing runs after a
# failure). PMC passes: one counter group per run, no tracing domains.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${ROUND:-r3}
O=gpurun_out/round
S=" ${STAGES:-tests bench prof} "
mkdir -p $O/pmc
K='k_render_fast<false|k_render_lean|k_render_gen|k_render_mix1|k_frame_'
run() { echo "== $*" >&2; "$@"; }
ok=0
if [[ $S == *" tests "* ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 200 --timeout-method thread ${TESTS:-} > $O/tests.log 2>&1 || ok=1
  tail -3 $O/tests.log
fi
[ $ok = 0 ] && [[ $S == *" bench "* ]] && {
  timeout -k 10 600 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || ok=1; cat $O/bench_c3.json; }
[ $ok = 0 ] && [[ $S == *" configs "* ]] && {
  timeout -k 10 300 python bench.py --config C2 > $O/bench_c2.json 2> $O/bench_c2.err && \
  timeout -k 10 600 python bench.py --config C4 --steps 3 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err && \
  timeout -k 10 900 python bench.py --config C5 --steps 2 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || ok=1; }
[ $ok = 0 ] && [[ $S == *" prof "* ]] && {
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o $R -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $O/bench_prof.json 2> $O/prof.err || ok=1; }
[ $ok = 0 ] && [[ $S == *" pmc "* ]] && {
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $O/pmc/fetch -o p -f csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu > /dev/null 2> $O/pmc_fetch.err && \
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $O/pmc/write -o p -f csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu > /dev/null 2> $O/pmc_write.err && \
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "$K" -d $O/pmc/sq -o p -f csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu > /dev/null 2> $O/pmc_sq.err || ok=1; }
echo rc=$ok
exit $ok
