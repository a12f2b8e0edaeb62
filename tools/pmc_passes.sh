#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, kernel-trace only; no
# sys/runtime traces beside --pmc) over a command given as arguments, e.g.
#   bash tools/pmc_passes.sh python -u bench.py --steps 20 --warmup 5 --no-nll --no-cpu
# Outputs gpurun_out/pmc/<pass>/..._counter_collection.csv
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="${PMC_OUT:-gpurun_out/pmc}"
mkdir -p "$OUT"
run() {
  local name="$1"; shift
  local counters="$1"; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $counters --output-format csv -d "$OUT/$name" -o run -- "$@" \
    > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
run fetch "FETCH_SIZE" "$@" &&
run write "WRITE_SIZE GRBM_GUI_ACTIVE" "$@" &&
run sq1 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" "$@" &&
run sq2 "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES" "$@"
