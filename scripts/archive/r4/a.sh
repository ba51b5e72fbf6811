#!/bin/bash
# round 4, first box: full GPU suite (incl. the new owner-shard and 2-rank tests), the 2-rank
# rehearsal of the N > 1 bench on one GPU (shard_parity / value_strong), a short N = 1 bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4a; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
IA_TEST_SHARE_GPU=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 450 --timeout-method thread > $O/pytest_multirank_share.log 2>&1 || { echo "multirank rehearsal failed"; tail -40 $O/pytest_multirank_share.log; exit 1; }
tail -1 $O/pytest_multirank_share.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --cpu-seconds 10 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
IA_BENCH_SHARE_GPU=1 IA_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 > $O/n2_owner.json 2> $O/n2_owner.err || { echo "n2 owner failed"; tail -30 $O/n2_owner.err; exit 1; }
cat $O/n2_owner.json
echo ALL-OK
