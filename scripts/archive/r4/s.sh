#!/bin/bash
# the strong-scaling emulation of one cfg3 job on the final round-4 kernels (row-interleaved
# split; DB-shard exchange traces)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4s; mkdir -p $O
timeout -k 10 400 python -u tools/strong_model.py 3 1 2 4 8 > $O/strong_rows.jsonl 2> $O/strong_rows.err || { echo "strong model failed"; tail $O/strong_rows.err; exit 1; }
cat $O/strong_rows.jsonl
for W in 1 2 4 8; do
  a="--pipeline 0"; [ $W -gt 1 ] && a="--pipeline 0 --shard-emulate $W --shard-jobs 1 --exchange peer"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/sh$W -o run -- python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline $a > $O/sh$W.log 2>&1 || { echo "trace W=$W failed"; tail $O/sh$W.log; exit 1; }
done
python3 tools/shard_model.py $O/sh1/run_kernel_trace.csv 1 3 > $O/shard_w1.txt 2>&1 || true
B1=$(python3 -c "import re;print(re.search(r'modelled ([\d.]+) ms per rank', open('$O/shard_w1.txt').read()).group(1))" || echo 0)
for W in 2 4 8; do python3 tools/shard_model.py $O/sh$W/run_kernel_trace.csv $W 3 $B1 $O/shard_w1.txt > $O/shard_w$W.txt 2>&1 || true; done
tail -3 $O/shard_w*.txt
rm -rf $O/sh1 $O/sh2 $O/sh4 $O/sh8
echo ALL-OK
