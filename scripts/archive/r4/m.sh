#!/bin/bash
# fused merge + gather phase stamps (diagnostic build PROBE=8: one sampled wave every 256 steps),
# sequential and pipelined cfg3
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4m; mkdir -p $O
for p in 0 1; do
  IA_LIBIA=image-analogies-python_amd/libia_probe8.so timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --pipeline $p > $O/probe_p$p.txt 2> $O/probe_p$p.err || { echo "probe $p failed"; tail -20 $O/probe_p$p.err; exit 1; }
  grep -c GSTAMP $O/probe_p$p.txt
done
echo ALL-OK
