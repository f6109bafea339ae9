# C3 bench: memory-instruction PMC pass (scratch attribution of WRITE_SIZE), then the C2
# diagnostic A/B (object-binned batch parts switched off; wrong images, timing only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/extra
mkdir -p $O
K='k_render_fast<false|k_render_lean|k_render_gen|k_render_mix1|k_frame_'
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_ANY --kernel-include-regex "$K" -d $O/pmc_mem -o p -f csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu > /dev/null 2> $O/pmc_mem.err || exit 1
VARIANTS="default obNOSHADOW obNOCAM" SCENES="boxes2:1920x1080:8" REPS=2 bash tools/gpu_ab_scenes.sh || exit 1
