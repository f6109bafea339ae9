# Round-end measurement: GPU tests, the C3 bench line, the config lines, the
# kernel trace and PMC passes (tools/gpu_round.sh), then the torchrun path at
# world size 1 (the distributed code of bench.py: bands + RCCL gather).
set -o pipefail
STAGES="tests bench configs prof pmc" bash tools/gpu_round.sh || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 1 --steps 5 --warmup 2 --no-cpu > gpurun_out/round/bench_torchrun1.json 2> gpurun_out/round/bench_torchrun1.err || exit 1
cat gpurun_out/round/bench_torchrun1.json
