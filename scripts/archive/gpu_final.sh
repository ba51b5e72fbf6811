#!/bin/bash
# One GPU-box session for the round's evidence: parity suite + smoke, PMC traffic of the dominant
# kernel (cfg3, cfg4), the bench lines (cfg3 with the CPU baseline, cfg4, cfg5) and the rocprofv3
# kernel trace + stats of the cfg3 command, all into gpurun_out/final/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
F=gpurun_out/${FINAL_DIR:-final}
mkdir -p $F
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $F/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $F/pytest_gpu.log; exit 1; }
tail -1 $F/pytest_gpu.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $F/smoke.log; exit 1; }
cat $F/smoke.log
timeout -k 10 300 bash tools/pmc_k3p.sh $F/pmc_cfg3 cfg3 k3h_prune3 --pipeline 0 > $F/pmc_cfg3.log 2>&1 || { echo "pmc cfg3 failed"; tail $F/pmc_cfg3.log; exit 1; }
python3 tools/k3p_traffic.py $F/pmc_cfg3 $F/k3p_traffic_cfg3.json cfg3 4093 > $F/k3p_traffic_cfg3.txt 2>&1 || { echo "traffic cfg3 failed"; exit 1; }
timeout -k 10 500 bash tools/pmc_k3p.sh $F/pmc_cfg4 cfg4 k3h_prune3 --pipeline 0 > $F/pmc_cfg4.log 2>&1 || { echo "pmc cfg4 failed"; tail $F/pmc_cfg4.log; exit 1; }
python3 tools/k3p_traffic.py $F/pmc_cfg4 $F/k3p_traffic_cfg4.json cfg4 8189 > $F/k3p_traffic_cfg4.txt 2>&1 || { echo "traffic cfg4 failed"; exit 1; }
cp $F/k3p_traffic_cfg3.json $F/k3p_traffic_cfg4.json profiles/   # the bench lines below read them
rm -rf $F/pmc_cfg3 $F/pmc_cfg4
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --cpu-seconds 20 > $F/bench.json 2> $F/bench.err || { echo "bench failed"; tail -20 $F/bench.err; exit 1; }
cut -c1-300 $F/bench.json
timeout -k 10 300 python -u bench.py --config cfg4 --steps 2 --warmup 1 --no-cpu-baseline > $F/bench_cfg4.json 2> $F/bench_cfg4.err || { echo "cfg4 failed"; tail -20 $F/bench_cfg4.err; exit 1; }
timeout -k 10 300 python -u bench.py --config cfg5 --steps 1 --warmup 1 --no-cpu-baseline > $F/bench_cfg5.json 2> $F/bench_cfg5.err || { echo "cfg5 failed"; tail -20 $F/bench_cfg5.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $F/prof.log 2>&1 || { echo "rocprof failed"; tail $F/prof.log; exit 1; }
cp /tmp/prof/run_kernel_stats.csv $F/kernel_stats.csv
python3 tools/trace_breakdown.py /tmp/prof/run_kernel_trace.csv 1 > $F/breakdown.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof0 -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --pipeline 0 > $F/prof_seq.log 2>&1 || { echo "rocprof seq failed"; tail $F/prof_seq.log; exit 1; }
cp /tmp/prof0/run_kernel_stats.csv $F/kernel_stats_seq.csv
python3 tools/trace_breakdown.py /tmp/prof0/run_kernel_trace.csv 1 > $F/breakdown_seq.txt 2>&1 || true
echo FINAL-OK
