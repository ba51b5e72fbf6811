#!/bin/bash
# round 3, session L: the driver's N = 2 bench path on one GPU (ranks on CU halves): owner
# exchange, and the agreed fallback to replicas when one rank's shard setup fails
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/l
export IA_BENCH_SHARE_GPU=1 IA_BENCH_BACKEND=gloo
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/l/n2_owner.json 2> gpurun_out/l/n2_owner.err || { echo "n2 owner failed"; tail -20 gpurun_out/l/n2_owner.err; exit 1; }
cut -c1-250 gpurun_out/l/n2_owner.json
IA_BENCH_FAIL_SHARD=1 timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/l/n2_fallback.json 2> gpurun_out/l/n2_fallback.err || { echo "n2 fallback failed"; tail -20 gpurun_out/l/n2_fallback.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/l/n2_fallback.json').read().strip().splitlines()[-1]); print('fallback', d['value'], d['config']['mode'], d['config'].get('shard_error'))"
echo R3L-OK
