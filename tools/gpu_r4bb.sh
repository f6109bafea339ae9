# Round 4 end check: smoke(), the driver's bench command, the torchrun path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4bb}
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
cut -c1-240 $O/bench.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu > $O/torchrun1.json 2> $O/torchrun1.err || { tail $O/torchrun1.err; exit 1; }
cut -c1-240 $O/torchrun1.json
grep -o '"frame_check": [^,]*' $O/torchrun1.json || true
