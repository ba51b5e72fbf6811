#!/bin/bash
# Same-box kernel traces of the pruned-scan variants (cfg3 and cfg4): 14 (hi x hi filter, then
# full chains), 18 (fused corrections, pipelined single chains), 20 (fused corrections on
# query-tile pairs), 11 (no filter).  Per-level breakdown into gpurun_out/var/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/var
prof() {  # tag config variant
  local tag=$1 cfg=$2 v=$3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$tag -o run -- python3 -u bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline --k3p-variant $v > gpurun_out/var/$tag.json 2> gpurun_out/var/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/var/$tag.err; return 1; }
  cp /tmp/$tag/run_kernel_stats.csv gpurun_out/var/$tag.csv
  python3 tools/trace_breakdown.py /tmp/$tag/run_kernel_trace.csv 1 > gpurun_out/var/$tag.txt 2>&1
  rm -rf /tmp/$tag
  echo "$tag: $(grep -E 'k3h_prune.*finest' gpurun_out/var/$tag.txt | cut -c1-90) | $(grep -E '^total' gpurun_out/var/$tag.txt | cut -c1-40)"
}
for v in 14 18 20; do prof cfg3_v$v cfg3 $v || exit 1; done
for v in 14 18 20 11; do prof cfg4_v$v cfg4 $v || exit 1; done
echo VAR-OK
