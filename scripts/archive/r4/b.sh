#!/bin/bash
# same-box A/B: fused sort on / off (interleaved), then a kernel trace of the default bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4b; mkdir -p $O
for i in 1 2; do
  for fs in 1 0; do
    timeout -k 10 200 python -u bench.py --steps 8 --warmup 1 --no-cpu-baseline --fuse-sort $fs > $O/fs${fs}_$i.json 2> $O/fs${fs}_$i.err || { echo "bench fs=$fs failed"; tail -20 $O/fs${fs}_$i.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/fs${fs}_$i.json'));r=d['roofline'];print('fs=$fs', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms', 'k3p', round(r.get('k3_us_per_launch_timed',0),2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'fallbacks', d['stats']['fallbacks'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
python3 tools/trace_breakdown.py $O/prof/run_kernel_trace.csv 1 > $O/breakdown.txt 2>&1 || true
python3 tools/pipe_trace.py $O/prof/run_kernel_trace.csv > $O/pipe_trace.txt 2>&1 || true
echo ALL-OK
