# C2 (boxes2 1080p/64 spp) issue profile: kernel trace + one SQ counter pass
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c2pmc
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/c2pmc/trace -o run -- python bench.py --config C2 --steps 5 --warmup 2 --no-cpu > gpurun_out/c2pmc/bench.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d gpurun_out/c2pmc/sq -o run -- python bench.py --config C2 --steps 2 --warmup 1 --no-cpu > gpurun_out/c2pmc/pmc.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_INSTS_SENDMSG -d gpurun_out/c2pmc/sq2 -o run -- python bench.py --config C2 --steps 2 --warmup 1 --no-cpu > gpurun_out/c2pmc/pmc2.log 2>&1 || exit 1
