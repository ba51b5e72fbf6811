#!/bin/bash
# round-5 baseline on this round's box: the default bench line, the sequential (one-stream) line,
# and the K3p phase probe (PROBE=16 build) of the sequential job
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${R5_OUT:-r5a}; mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --pipeline 0 > $O/bench_seq.json 2> $O/bench_seq.err || { echo "bench seq failed"; tail -20 $O/bench_seq.err; exit 1; }
IA_LIBIA=$PWD/image-analogies-python_amd/libia_probe16.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --pipeline 0 > $O/probe.json 2> $O/probe.err || { echo "probe failed"; tail -20 $O/probe.err; exit 1; }
grep K3P_PROBE $O/probe.err | tail -8
for f in bench bench_seq; do
python3 -c "
import json; d=json.load(open('$O/$f.json')); r=d['roofline']
print('$f', round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms', 'frac_timed', round(r['frac_timed'],3), 'k3p', round(r['k3_us_per_launch_timed'],2), 'wg', round(r['k3_wg_us_timed'],2), 'spread', round(r['k3_start_spread_us_timed'],2), 'merge', round(r.get('merge_us_per_launch_timed',0),2), 'gap', round(r.get('chain_gap_us_timed',0),2), 'win', round(r.get('chain_window_ms_timed',0),1))"
done
echo ALL-OK
