set -o pipefail
cd $GRAFT_REPO_ROOT
L=$(ls $PWD/tools/ab/*.so | tr "\n" "," | sed "s/,$//")
RTMI_LIBS=$L ABLATE=c3_full REPS=8 timeout -k 10 300 python tools/ab.py 2>&1 | grep -v stats | grep -v amdgpu.ids || exit 1
RTMI_NO_SHADOW_LISTS=1 RTMI_LIBS=$L ABLATE=c3_full REPS=8 timeout -k 10 300 python tools/ab.py 2>&1 | grep -v stats | grep -v amdgpu.ids
