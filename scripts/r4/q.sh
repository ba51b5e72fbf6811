#!/bin/bash
# nn_bound on owner-computes (exchange 2) levels: the emulated-shard tests, the two-rank
# rehearsal on one GPU (CU halves), and the N = 2 bench line (rehearsal) with its parity checks
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4q; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread > $O/pytest_shard.log 2>&1 || { echo "shard tests failed"; tail -40 $O/pytest_shard.log; exit 1; }
tail -1 $O/pytest_shard.log
IA_TEST_SHARE_GPU=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 500 --timeout-method thread > $O/pytest_multirank.log 2>&1 || { echo "multirank failed"; tail -40 $O/pytest_multirank.log; exit 1; }
tail -3 $O/pytest_multirank.log
IA_BENCH_SHARE_GPU=1 IA_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_n2.json 2> $O/bench_n2.err || { echo "bench n2 failed"; tail -30 $O/bench_n2.err; exit 1; }
python3 -c "
import json; d=[json.loads(l) for l in open('$O/bench_n2.json') if l.startswith('{')][0]
print({k: d.get(k) for k in ('value','value_replicas','value_strong','shard_parity','strong_parity','ms_per_step')})"
echo ALL-OK
