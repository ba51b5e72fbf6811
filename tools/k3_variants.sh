#!/bin/bash
# bench every K3h schedule variant (records must be identical: same stats) + kernel stats
set -o pipefail
OUT=${1:-gpurun_out/var}; mkdir -p "$OUT"
for v in ${VARIANTS:-0 1 2 3}; do
  timeout -k 10 200 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --k3-variant $v > "$OUT/bench_v$v.json" 2> "$OUT/bench_v$v.err" || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in ${VARIANTS:-0 1 2 3}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_v$v" -o run -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --time-stride 0 --k3-variant $v > "$OUT/prof_v$v.log" 2>&1 || exit 1
done
echo VAR-OK
