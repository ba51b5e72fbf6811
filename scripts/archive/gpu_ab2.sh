#!/bin/bash
# Same-box A/B of the cfg3 bench line: this tree vs ab_base (a worktree of the last commit with
# its own libia.so), alternated three times, plus one rocprofv3 breakdown of each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab2
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab2/head_$i.json 2> gpurun_out/ab2/head_$i.err || { echo "head bench failed"; exit 1; }
  (cd ab_base && timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > ../gpurun_out/ab2/base_$i.json 2> ../gpurun_out/ab2/base_$i.err) || { echo "base bench failed"; exit 1; }
done
for f in gpurun_out/ab2/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(round(d['value']), round(d['ms_per_step'],1), round(d['roofline'].get('k3_us_per_launch',0),1))")"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab2/prof_head -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 1
python3 tools/trace_breakdown.py gpurun_out/ab2/prof_head/run_kernel_trace.csv 1 > gpurun_out/ab2/breakdown_head.txt 2>&1
(cd ab_base && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ../gpurun_out/ab2/prof_base -o run -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2>&1) || exit 1
python3 tools/trace_breakdown.py gpurun_out/ab2/prof_base/run_kernel_trace.csv 1 > gpurun_out/ab2/breakdown_base.txt 2>&1
grep finest gpurun_out/ab2/breakdown_head.txt; echo base; grep finest gpurun_out/ab2/breakdown_base.txt
echo ALL-OK
