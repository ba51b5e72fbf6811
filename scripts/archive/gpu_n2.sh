#!/bin/bash
# Rehearsal of the driver's N > 1 bench path on a one-GPU box: two replica ranks sharing GPU 0
# over gloo (barrier, max-over-ranks time, rank-0 JSON line), cfg3 and cfg5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out/n2
export IA_BENCH_SHARE_GPU=1 IA_BENCH_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/n2/cfg3.json 2> gpurun_out/n2/cfg3.err || { echo "n2 cfg3 failed"; tail -20 gpurun_out/n2/cfg3.err; exit 1; }
cat gpurun_out/n2/cfg3.json | cut -c1-400
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/n2/cfg5.json 2> gpurun_out/n2/cfg5.err || { echo "n2 cfg5 failed"; tail -20 gpurun_out/n2/cfg5.err; exit 1; }
cat gpurun_out/n2/cfg5.json | cut -c1-400
echo N2-OK
