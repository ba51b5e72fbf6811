#!/bin/bash
# rocprofv3 kernel stats of one bench configuration (extra bench args in $@); only the stats
# CSV and a per-level breakdown come back (full traces exceed the copy-back limit).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
TAG=${TAG:-prof}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$TAG -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { echo "rocprof failed"; tail -20 gpurun_out/$TAG/bench.err; exit 1; }
cp /tmp/$TAG/run_kernel_stats.csv gpurun_out/$TAG/kernel_stats.csv
python3 tools/trace_breakdown.py /tmp/$TAG/run_kernel_trace.csv 1 > gpurun_out/$TAG/breakdown.txt 2>&1 || true
cut -c1-300 gpurun_out/$TAG/bench.json
tail -3 gpurun_out/$TAG/breakdown.txt
