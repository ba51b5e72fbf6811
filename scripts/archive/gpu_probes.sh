#!/bin/bash
# Same-box kernel profiles of the pruned-scan variants and diagnostic builds (timing only):
# v7, v14 (hi x hi block filter), v14 never-pass (PROBE=64), v14 always-pass (PROBE=128),
# after the exactness tests of the variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out/probes
timeout -k 10 400 python -u -m pytest tests/test_gpu_prune.py tests/test_gpu_batch.py -m gpu -x -v --timeout 300 --timeout-method thread -k "14 or 15 or wide" > gpurun_out/probes/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/probes/pytest.log; exit 1; }
tail -1 gpurun_out/probes/pytest.log; grep -h "corrected pairs" gpurun_out/probes/pytest.log | head -4
prof() {  # tag lib extra-args...
  local tag=$1 lib=$2
  shift 2
  IA_LIBIA=$R/image-analogies-python_amd/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/$tag -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/probes/$tag.json 2> gpurun_out/probes/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/probes/$tag.err; return 1; }
  python3 tools/trace_breakdown.py /tmp/$tag/run_kernel_trace.csv 1 > gpurun_out/probes/$tag.txt 2>&1
  rm -rf /tmp/$tag
  echo "$tag: $(grep -E 'k3h_prune finest' gpurun_out/probes/$tag.txt | head -1 | cut -c1-160)"
}
for v in ${VARIANTS:-v7 v14 v14_never v14_always}; do
  case $v in
    v7) prof v7 libia.so ;;
    v14) prof v14 libia.so --k3p-variant 14 ;;
    v14_never) prof v14_never libia_probe64.so --k3p-variant 14 ;;
    v14_always) prof v14_always libia_probe128.so --k3p-variant 14 ;;
  esac || exit 1
done
echo ALL-OK
