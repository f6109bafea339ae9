# Round 4 measurement: the GPU suite, the C3 bench line + kernel trace, the
# config lines, then the PMC passes of every config (tools/gpu_pmc_configs.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
ROUND=r4 STAGES="tests bench configs prof" bash tools/gpu_round.sh || exit 1
CONFIGS="C3 C2 C4 C5" bash tools/gpu_pmc_configs.sh || exit 1
