set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r1 -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/bench_prof.json 2> gpurun_out/prof.err
