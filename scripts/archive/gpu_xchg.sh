#!/bin/bash
# Peer-write exchange: emulated shards (pytest), the two-process IPC rehearsal on one GPU, the
# bench's N = 2 shard path rehearsed with both ranks on GPU 0, then the N = 1 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_shard.log 2>&1 || { echo "shard tests failed"; tail -40 gpurun_out/pytest_shard.log; exit 1; }
tail -1 gpurun_out/pytest_shard.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 tools/xchg_rehearsal.py > gpurun_out/xchg_rehearsal.log 2>&1 || { echo "rehearsal failed"; tail -30 gpurun_out/xchg_rehearsal.log; exit 1; }
grep -E "rank|XCHG" gpurun_out/xchg_rehearsal.log
IA_BENCH_SHARE_GPU=1 IA_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 2 --warmup 1 > gpurun_out/bench_n2_shard.json 2> gpurun_out/bench_n2_shard.err || { echo "n2 bench failed"; tail -30 gpurun_out/bench_n2_shard.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_n2_shard.json')); print('n2 shard', round(d['value']), 'replicas', round(d.get('value_replicas') or 0), d['config']['parallelism'], d['config']['exchange'])"
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
echo XCHG-OK
