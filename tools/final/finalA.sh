set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${OUT:-r6fa}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_px64.py tests/test_gpu_reference_inputs.py -m gpu -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { tail $O/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c3.json'));print('C3', d['value'], d['ms_per_step'], d['fp64_parity']['ms_per_step'], d['bvh_path']['ms_per_step'])"
for c in C2 BVHMIX; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail $O/bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c', d['value'], d['ms_per_step'])"
done
for c in C4 C5; do
  timeout -k 10 600 python bench.py --config $c --steps 5 --warmup 1 --no-cpu > $O/bench_$c.json 2> $O/bench_$c.err || { tail $O/bench_$c.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$c.json'));print('$c', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o p -f csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu > $O/prof_c3.json 2> $O/prof_c3.err || { tail $O/prof_c3.err; exit 1; }
echo finalA ok
