# Full measurement pass for one round (ROUND=r2): GPU tests, bench lines for
# every BASELINE config, rocprofv3 kernel trace + stats of the C3 bench, and
# the PMC passes (FETCH_SIZE, WRITE_SIZE, SQ instruction mix) of the render
# call's kernels, each counter group in its own pass (no tracing domains with
# --pmc). Outputs under gpurun_out/round/ (copied into profiles/ afterwards).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${ROUND:-r2}
O=gpurun_out/round
mkdir -p $O/pmc
K='k_render_fast<false|k_render_lean|k_render_gen|k_render_mix1'
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 && \
timeout -k 10 600 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err && \
timeout -k 10 300 python bench.py --config C2 > $O/bench_c2.json 2> $O/bench_c2.err && \
timeout -k 10 600 python bench.py --config C4 --steps 3 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err && \
timeout -k 10 900 python bench.py --config C5 --steps 2 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o $R -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $O/bench_prof.json 2> $O/prof.err && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d $O/pmc/fetch -o p -f csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu > /dev/null 2> $O/pmc_fetch.err && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d $O/pmc/write -o p -f csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu > /dev/null 2> $O/pmc_write.err && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "$K" -d $O/pmc/sq -o p -f csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu > /dev/null 2> $O/pmc_sq.err
rc=$?
tail -2 $O/tests.log
echo rc=$rc
exit $rc
