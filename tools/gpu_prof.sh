# Full measurement pass for one round: bench line, rocprofv3 kernel trace +
# stats, and the PMC passes (FETCH_SIZE, WRITE_SIZE, SQ instruction mix) for
# the render kernel, each counter group in its own pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
K='k_render_fast<false>'
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r1 -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_prof.json 2> gpurun_out/prof.err && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" -d gpurun_out/pmc/fetch -o p -f csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu > /dev/null 2> gpurun_out/pmc/fetch.err && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" -d gpurun_out/pmc/write -o p -f csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu > /dev/null 2> gpurun_out/pmc/write.err && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "$K" -d gpurun_out/pmc/sq -o p -f csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu > /dev/null 2> gpurun_out/pmc/sq.err
