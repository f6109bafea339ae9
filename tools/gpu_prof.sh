# Full measurement pass for one round: GPU tests, bench lines for every
# BASELINE config, rocprofv3 kernel trace + stats of the C3 bench, and the PMC
# passes (FETCH_SIZE, WRITE_SIZE, SQ instruction mix) for the render kernel,
# each counter group in its own pass (no tracing domains with --pmc).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc gpurun_out/round
K='k_render_fast<false'
O=gpurun_out/round
timeout -k 10 700 python -m pytest tests -m gpu -q > $O/tests.log 2>&1 && \
timeout -k 10 600 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err && \
timeout -k 10 300 python bench.py --config C2 > $O/bench_c2.json 2> $O/bench_c2.err && \
timeout -k 10 600 python bench.py --config C4 --steps 3 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err && \
timeout -k 10 900 python bench.py --config C5 --steps 2 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r1 -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $O/bench_prof.json 2> $O/prof.err && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d gpurun_out/pmc/fetch -o p -f csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu > /dev/null 2> gpurun_out/pmc/fetch.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d gpurun_out/pmc/write -o p -f csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu > /dev/null 2> gpurun_out/pmc/write.err && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "$K" -d gpurun_out/pmc/sq -o p -f csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu > /dev/null 2> gpurun_out/pmc/sq.err
rc=$?
tail -2 $O/tests.log
echo rc=$rc
exit $rc
