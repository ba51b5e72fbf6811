#!/bin/bash
# round 3, session U: kernel traces of the pipelined job with 2 and 4 contexts (tools/pipe_trace.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/u
for c in ${CTXS:-4 2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pt$c -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --pipe-ctx $c --pipe-priority 1 > gpurun_out/u/trace_c$c.json 2> gpurun_out/u/trace_c$c.err || { echo "trace $c failed"; tail -5 gpurun_out/u/trace_c$c.err; exit 1; }
  python3 tools/pipe_trace.py /tmp/pt$c/run_kernel_trace.csv > gpurun_out/u/pipe_c$c.txt 2>&1
  cat gpurun_out/u/pipe_c$c.txt
  gzip -c /tmp/pt$c/run_kernel_trace.csv > gpurun_out/u/trace_c$c.csv.gz
  rm -rf /tmp/pt$c
done
echo R3U-OK
