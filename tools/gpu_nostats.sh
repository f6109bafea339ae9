set -o pipefail
cd $GRAFT_REPO_ROOT
for f in 0 0x200 0 0x200; do
  RTMI_FLAGS=$f REPS=7 timeout -k 10 120 python tools/time_c3.py | cut -c1-100 || exit 1
  RTMI_FLAGS=$f BANDS=4 REPS=5 timeout -k 10 200 python tools/scaling_sim.py | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: v for k, v in d.items() if 'max' in k or 'speed' in k})" || exit 1
done
