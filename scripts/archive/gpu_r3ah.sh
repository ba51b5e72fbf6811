#!/bin/bash
# round 3, session AH: rocprofv3 kernel stats of the cfg4 and cfg5 bench commands (final build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ah
for cfg in cfg4 cfg5; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p$cfg -o run -- python3 -u bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/ah/$cfg.json 2> gpurun_out/ah/$cfg.err || { echo "$cfg failed"; tail -5 gpurun_out/ah/$cfg.err; exit 1; }
  cp /tmp/p$cfg/run_kernel_stats.csv gpurun_out/ah/kernel_stats_$cfg.csv
  python3 tools/trace_breakdown.py /tmp/p$cfg/run_kernel_trace.csv 1 > gpurun_out/ah/breakdown_$cfg.txt 2>&1 || true
  rm -rf /tmp/p$cfg
  head -4 gpurun_out/ah/kernel_stats_$cfg.csv | cut -c1-160
done
echo R3AH-OK
