set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
export OUT=${OUT:-r6fc}
STAGES="pmc:C4 pmc:C5" bash tools/gpu_job.sh || exit 1
O=gpurun_out/$OUT
for c in C3 C4 C5; do
  R=20; [ $c = C5 ] && R=6; [ $c = C4 ] && R=10
  CONFIG=$c REPS=$R timeout -k 10 600 python tools/scaling_sim.py > $O/scaling_$c.json 2> $O/scaling_$c.err || { tail $O/scaling_$c.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/scaling_$c.json').readline());print('$c', d['step1_ms'], [d.get('projected_speedup_%d'%n) for n in (2,4,8)])"
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu > $O/bench_c3_torchrun1.json 2> $O/torchrun1.err || { tail -20 $O/torchrun1.err; exit 1; }
echo finalC ok
