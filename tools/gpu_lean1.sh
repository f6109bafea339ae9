# split/parity/bins GPU tests, C3 timing, band-launch scaling projection (mix on / off)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/lean1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_bins.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for m in 1 0; do
RTMI_MIX=$m REPS=7 timeout -k 10 120 python tools/time_c3.py | cut -c1-100 || exit 1
RTMI_MIX=$m BANDS=4 REPS=5 timeout -k 10 200 python tools/scaling_sim.py | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: v for k, v in d.items() if 'max' in k or 'speed' in k})" || exit 1
done
