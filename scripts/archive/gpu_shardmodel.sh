#!/bin/bash
# DESIGN §7 cost model inputs: cfg3 with W emulated DB shards on one GPU and W jobs stepped
# together (bench.py's N > 1 shard mode; peer-write exchange kernels, all W shards' scans and
# publishes back to back, then the finishing merge), one rocprofv3 kernel trace each; per-level /
# per-kernel breakdown and the per-rank model into gpurun_out/shard/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/shard
for W in ${WS:-1 2 4 8}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/sh$W -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --shard-emulate $W --shard-jobs $W --exchange ${EXCH:-owner} > gpurun_out/shard/w$W.json 2> gpurun_out/shard/w$W.err || { echo "W=$W failed"; tail -5 gpurun_out/shard/w$W.err; exit 1; }
  cp /tmp/sh$W/run_kernel_stats.csv gpurun_out/shard/w${W}_stats.csv
  python3 tools/trace_breakdown.py /tmp/sh$W/run_kernel_trace.csv 1 > gpurun_out/shard/w$W.txt 2>&1
  B1=profiles/r03/shard_jobs/w1_model.txt; [ -f gpurun_out/shard/w1_model.txt ] && B1=gpurun_out/shard/w1_model.txt
  # baseline: the W = 1 run's modelled job time (one job alone, same kernels)
  B0=$(grep -oP 'modelled \K[0-9.]+' gpurun_out/shard/w1_model.txt 2>/dev/null || echo 382)
  python3 tools/shard_model.py /tmp/sh$W/run_kernel_trace.csv $W 3.0 $B0 $B1 > gpurun_out/shard/w${W}_model.txt 2>&1 || true
  rm -rf /tmp/sh$W
  grep -E "^level 9|^total" gpurun_out/shard/w$W.txt | cut -c1-400
  cat gpurun_out/shard/w${W}_model.txt
done
echo SHARD-OK
