set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${OUT:-r6gD}; mkdir -p $O
timeout -k 10 400 python bench.py > $O/bench_c3.json 2> $O/bench_c3.err || { tail $O/bench_c3.err; exit 1; }
for c in C2 BVHMIX; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail $O/bench_$c.err; exit 1; }
done
for c in C4 C5; do
  timeout -k 10 600 python bench.py --config $c --steps 5 --warmup 1 --no-cpu > $O/bench_$c.json 2> $O/bench_$c.err || { tail $O/bench_$c.err; exit 1; }
done
for f in $O/bench_*.json; do python -c "
import json;d=json.load(open('$f'));r=d['roofline'];print('$f', d['value'], d['ms_per_step'], r.get('frac'), r.get('frac_net_of_spills_est'), r.get('traffic'))"; done
echo finalD ok
