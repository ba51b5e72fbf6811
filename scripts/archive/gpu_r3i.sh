#!/bin/bash
# round 3, session I: owner-computes sharded steps (exchange = 2): shard tests, the two-process
# IPC rehearsal, the N = 2 bench path on one GPU, then the emulated cost model (W = 2, 4, 8)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/i
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py -x -v -k "owner or batched" --timeout 300 --timeout-method thread > gpurun_out/i/pytest.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/i/pytest.log; exit 1; }
tail -3 gpurun_out/i/pytest.log
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 tools/xchg_rehearsal.py > gpurun_out/i/xchg_rehearsal.log 2>&1 || { echo "rehearsal failed"; tail -30 gpurun_out/i/xchg_rehearsal.log; exit 1; }
grep -E "rank|XCHG" gpurun_out/i/xchg_rehearsal.log
IA_BENCH_SHARE_GPU=1 IA_BENCH_BACKEND=gloo timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/i/n2_owner.json 2> gpurun_out/i/n2_owner.err || { echo "n2 owner failed"; tail -20 gpurun_out/i/n2_owner.err; exit 1; }
cut -c1-300 gpurun_out/i/n2_owner.json
WS="2 4 8" bash scripts/gpu_shardmodel.sh || exit 1
echo R3I-OK
