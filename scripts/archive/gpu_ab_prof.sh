#!/bin/bash
# Same-box kernel profiles of this tree vs the round-2 start (ab_base worktree), plus the
# single-product diagnostic build (libia_probe32.so: K3p with only the hi x hi MFMA product).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out/abp
prof() {  # tag dir extra-args...
  local tag=$1 dir=$2
  shift 2
  (cd $dir && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$tag -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@" > $R/gpurun_out/abp/$tag.json 2> $R/gpurun_out/abp/$tag.err) || { echo "$tag failed"; tail -5 gpurun_out/abp/$tag.err; return 1; }
  cp /tmp/$tag/run_kernel_stats.csv gpurun_out/abp/$tag.csv
  python3 tools/trace_breakdown.py /tmp/$tag/run_kernel_trace.csv 1 > gpurun_out/abp/$tag.txt 2>&1
  rm -rf /tmp/$tag
  tail -12 gpurun_out/abp/$tag.txt | cut -c1-400
}
prof head . || exit 1
prof base ab_base || exit 1
prof head2 . || exit 1
prof base2 ab_base || exit 1
IA_LIBIA=$R/image-analogies-python_amd/libia_probe32.so prof probe32 . || exit 1
echo ALL-OK
