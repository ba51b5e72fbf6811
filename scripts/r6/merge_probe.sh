#!/bin/bash
# round 6: fused merge + gather phase stamps (make PROBE=8 -> libia_probe8.so), sequential and pipelined cfg3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/$1; L=${2:-libia_probe8.so}; mkdir -p $O
for mode in 0 1; do
  IA_LIBIA=$PWD/image-analogies-python_amd/$L timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --pipeline $mode > $O/bench_p$mode.json 2> $O/probe_p$mode.err || { echo "bench failed"; tail -20 $O/probe_p$mode.err; exit 1; }
  echo "pipeline $mode"; python3 tools/merge_probe.py $O/bench_p$mode.json
done
