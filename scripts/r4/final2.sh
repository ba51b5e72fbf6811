#!/bin/bash
# round-4 final evidence (nn_bound, k3p_variant 22, pruned 512^2 levels in the bench configs): GPU suite +
# the bench lines (cfg3 default, cfg4, cfg5) and the rocprofv3 kernel trace of the cfg3 command
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/r4final2; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 bash tools/pmc_k3p.sh $O/pmc3 cfg3 k3h_prune3 --pipeline 0 || exit 1
python3 tools/k3p_traffic.py $O/pmc3 profiles/k3p_traffic_cfg3.json cfg3 4093 > $O/traffic3.txt 2>&1 || { echo "traffic3 failed"; tail $O/traffic3.txt; exit 1; }
timeout -k 10 400 bash tools/pmc_k3p.sh $O/pmc4 cfg4 k3h_prune3 --pipeline 0 || exit 1
python3 tools/k3p_traffic.py $O/pmc4 profiles/k3p_traffic_cfg4.json cfg4 8189 > $O/traffic4.txt 2>&1 || { echo "traffic4 failed"; tail $O/traffic4.txt; exit 1; }
rm -rf $O/pmc3 $O/pmc4
timeout -k 10 400 python -u bench.py --steps 20 --warmup 2 > $O/bench_cfg3.json 2> $O/bench_cfg3.err || { echo "bench cfg3 failed"; tail -20 $O/bench_cfg3.err; exit 1; }
cat $O/bench_cfg3.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
python3 tools/trace_breakdown.py $O/prof/run_kernel_trace.csv 1 > $O/breakdown.txt 2>&1 || true
python3 tools/pipe_trace.py $O/prof/run_kernel_trace.csv > $O/pipe_trace.txt 2>&1 || true
cp $O/prof/run_kernel_stats.csv $O/kernel_stats.csv; rm -f $O/prof/run_kernel_trace.csv
timeout -k 10 400 python -u bench.py --config cfg4 --steps 3 --warmup 1 --cpu-seconds 15 > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { echo "bench cfg4 failed"; tail -20 $O/bench_cfg4.err; exit 1; }
timeout -k 10 400 python -u bench.py --config cfg5 --steps 3 --warmup 1 --cpu-seconds 15 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { echo "bench cfg5 failed"; tail -20 $O/bench_cfg5.err; exit 1; }
python3 -c "
import json
for c in ('cfg3','cfg4','cfg5'):
    d=json.load(open('$O/bench_%s.json'%c)); r=d['roofline']
    print(c, round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms', 'frac', round(r['frac'],3), 'frac_timed', round(r.get('frac_timed',0),3), 'k3p_timed', round(r.get('k3_us_per_launch_timed',0),2), 'traffic', r.get('traffic'))"
timeout -k 10 300 python -u tools/dump_state.py $O/cfg3_state.npz cfg3 5 6 7 8 9 > $O/dump3.log 2>&1 || { echo "dump cfg3 failed"; tail $O/dump3.log; exit 1; }
timeout -k 10 300 python -u tools/dump_state.py $O/cfg4_state.npz cfg4 > $O/dump4.log 2>&1 || { echo "dump cfg4 failed"; tail $O/dump4.log; exit 1; }
echo ALL-OK
