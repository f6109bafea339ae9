# Round 4: band height and lean lanes per pixel against the N = 8 projection.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4t}
mkdir -p $O
REPS=20 BANDS=2,4,8,16 timeout -k 10 400 python tools/scaling_sim.py > $O/ss_bands.jsonl 2> $O/ss.err || { tail $O/ss.err; exit 1; }
cat $O/ss_bands.jsonl
RTMI_LEAN_LP=4 REPS=20 BANDS=4 timeout -k 10 300 python tools/scaling_sim.py > $O/ss_lp4.json 2> $O/ss4.err || exit 1
echo lp4; cat $O/ss_lp4.json
