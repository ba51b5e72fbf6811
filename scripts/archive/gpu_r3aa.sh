#!/bin/bash
# round 3, session AA: owner-computes with the fused merge's waiter wave: shard parity tests, the
# N = 2 owner path on one GPU (IPC, ranks on CU halves) without and with pipelined levels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/aa
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shard.py > gpurun_out/aa/pytest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/aa/pytest.log; exit 1; }
tail -1 gpurun_out/aa/pytest.log
export IA_BENCH_SHARE_GPU=1 IA_BENCH_BACKEND=gloo
for op in 0 1; do
  timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2954$op bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --owner-pipeline $op > gpurun_out/aa/n2_op$op.json 2> gpurun_out/aa/n2_op$op.err || { echo "n2 op$op failed"; tail -20 gpurun_out/aa/n2_op$op.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/aa/n2_op$op.json').read().strip().splitlines()[-1]); print('op$op', round(d['value']), round(d['ms_per_step'],1), d['config'].get('level_pipeline'))"
done
echo R3AA-OK
