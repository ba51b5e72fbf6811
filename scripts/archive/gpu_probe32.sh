#!/bin/bash
# bf16 / single-product prefilter question: K3p of the product build vs the
# timing-only PROBE=32 build (libia_probe32.so: one f16 MFMA product per 16 k instead of three,
# results invalid) on cfg3 and cfg4, one rocprofv3 kernel trace each, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out/p32
prof() {  # tag config libia [bench args...]
  local tag=$1 cfg=$2 lib=$3
  shift 3
  IA_LIBIA=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$tag -o run -- python3 -u bench.py --config $cfg --steps 1 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/p32/$tag.json 2> gpurun_out/p32/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/p32/$tag.err; return 1; }
  cp /tmp/$tag/run_kernel_stats.csv gpurun_out/p32/$tag.csv
  python3 tools/trace_breakdown.py /tmp/$tag/run_kernel_trace.csv 1 > gpurun_out/p32/$tag.txt 2>&1
  rm -rf /tmp/$tag
  grep -E "k3h_prune.*finest|^total" gpurun_out/p32/$tag.txt | cut -c1-300
}
P32=$R/image-analogies-python_amd/libia_probe32.so
prof cfg3_prod cfg3 "" && prof cfg3_p32 cfg3 $P32 && prof cfg4_prod cfg4 "" && prof cfg4_p32 cfg4 $P32 &&
  prof cfg4_v11 cfg4 "" --k3p-variant 11 && prof cfg3_v11 cfg3 "" --k3p-variant 11 &&
  prof cfg3_v18 cfg3 "" --k3p-variant 18 && prof cfg4_v18 cfg4 "" --k3p-variant 18 && echo P32-OK
