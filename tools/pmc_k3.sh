#!/bin/bash
# PMC passes over the K3 distance kernel of one cfg3 bench step (run on the GPU box from the
# repo root).  One rocprofv3 run per counter group (gfx950 slot limits: 8 SQ, 4 TCC, 2 GRBM).
#   tools/pmc_k3.sh <out_dir> <k3_variant> [kernel_regex]
set -o pipefail
OUT=${1:-gpurun_out/pmc}; V=${2:-1}; RX=${3:-k3h_dist}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
BENCH="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --time-stride 0 --k3-variant $V"
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-include-regex "$RX" --output-format csv \
      -d "$OUT/$name" -o run -- $BENCH > "$OUT/$name.log" 2>&1 || { echo "pass $name failed rc=$?"; return 1; }
}
pass p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
        SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE &&
pass p2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES \
        SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE &&
pass p3 FETCH_SIZE &&
pass p4 WRITE_SIZE &&
echo PMC-OK
