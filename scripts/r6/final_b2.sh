#!/bin/bash
# round-6 final evidence, part B (after the PMC wait-ratio passes): cfg4's PMC traffic and bench
# line, cfg5's bench line, the teacher-forcing tests, the two-rank rehearsal on one GPU, the probe
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6final}; mkdir -p $O
timeout -k 10 400 bash tools/pmc_k3p.sh $O/pmc4 cfg4 k3h_prune3 --pipeline 0 || exit 1
python3 tools/k3p_traffic.py $O/pmc4 profiles/k3p_traffic_cfg4.json cfg4 8189 > $O/traffic4.txt 2>&1 || { echo "traffic4 failed"; tail $O/traffic4.txt; exit 1; }
cp profiles/k3p_traffic_cfg4.json $O/ ; rm -rf $O/pmc4
timeout -k 10 400 python -u bench.py --config cfg4 --steps 3 --warmup 1 --cpu-seconds 15 > $O/bench_cfg4.json 2> $O/bench_cfg4.err || { echo "bench cfg4 failed"; tail -20 $O/bench_cfg4.err; exit 1; }
timeout -k 10 400 python -u bench.py --config cfg5 --steps 3 --warmup 1 --cpu-seconds 15 > $O/bench_cfg5.json 2> $O/bench_cfg5.err || { echo "bench cfg5 failed"; tail -20 $O/bench_cfg5.err; exit 1; }
python3 -c "
import json
for c in ('cfg4','cfg5'):
    d=json.load(open('$O/bench_%s.json'%c)); r=d['roofline']
    print(c, round(d['value']/1e6,3), 'M px/s', round(d['ms_per_step'],1), 'ms', 'frac', round(r['frac'],3), 'frac_timed', round(r.get('frac_timed',0),3), 'k3p_timed', round(r.get('k3_us_per_launch_timed',0),2), 'traffic', r.get('traffic'), 'parity', d.get('parity'))"
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -x -v --timeout 500 --timeout-method thread -k "teacher_forced_1024 or teacher_forced_cfg4" --durations=0 > $O/pytest_teacher.log 2>&1 || { echo "teacher-forcing tests failed"; tail -30 $O/pytest_teacher.log; exit 1; }
grep -E "passed|failed|s call" $O/pytest_teacher.log | tail -4
IA_TEST_SHARE_GPU=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_multirank.py -x -q --timeout 240 --timeout-method thread > $O/pytest_multirank_share.log 2>&1 || { echo "multirank rehearsal failed"; tail -30 $O/pytest_multirank_share.log; exit 1; }
tail -1 $O/pytest_multirank_share.log
IA_LIBIA=$PWD/image-analogies-python_amd/libia_probe16.so timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --pipeline 0 > $O/probe.json 2> $O/probe.err || { echo "probe failed"; tail -20 $O/probe.err; exit 1; }
grep K3P_PROBE $O/probe.err | tail -7
echo ALL-OK
