# Round 4: float64 parity kernel skipping the traversals the pixel records
# prove empty: the bit-exact parity tests, then the fp64 C3 bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4x}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_dropin.py tests/test_gpu_frame.py tests/test_samplers.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python bench.py --precision fp64 --steps 3 --warmup 1 --no-cpu > $O/c3_fp64.json 2> $O/c3_fp64.err || exit 1
echo "fp64 $(grep -o '"value": [0-9.]*' $O/c3_fp64.json) $(grep -o '"ms_per_step": [0-9.]*' $O/c3_fp64.json)"
