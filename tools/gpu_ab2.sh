# A/B of tools/ab/*.so on C3 with the merged kernel and with separate kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
L=$(ls $PWD/tools/ab/*.so | tr "\n" "," | sed "s/,$//")
RTMI_LIBS=$L ABLATE=c3_full REPS=6 timeout -k 10 300 python tools/ab.py 2>&1 | grep -v stats | grep -v amdgpu.ids || exit 1
RTMI_MIX=0 RTMI_LIBS=$L ABLATE=c3_full REPS=6 timeout -k 10 300 python tools/ab.py 2>&1 | grep -v stats | grep -v amdgpu.ids
