#!/bin/bash
# PMC passes over the pruned distance kernel (k3h_prune3) of one cfg3 bench step, run on the GPU
# box from the repo root.  One rocprofv3 run per counter group (gfx950 limits: 8 SQ, 4 TCC,
# 2 GRBM per pass; FETCH_SIZE and WRITE_SIZE need a pass each).
#   tools/pmc_k3p.sh <out_dir> [config] [kernel_regex] [extra bench args...]
set -o pipefail
OUT=${1:-gpurun_out/pmc_k3p}
CFG=${2:-cfg3}
RX=${3:-k3h_prune3}
shift 3 2>/dev/null || shift $#
EXTRA="$*"
mkdir -p "$OUT"
export TMPDIR=/tmp
pass() {  # name counters...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "$RX" --output-format csv \
      -d "$OUT/$name" -o run -- python3 bench.py --config "$CFG" --steps 1 --warmup 0 --no-cpu-baseline --time-stride 0 $EXTRA \
      > "$OUT/$name.log" 2>&1 || { echo "pass $name failed rc=$?"; tail -5 "$OUT/$name.log"; return 1; }
}
pass fetch FETCH_SIZE &&
pass write WRITE_SIZE &&
pass sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES \
        SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE &&
echo PMC-OK
