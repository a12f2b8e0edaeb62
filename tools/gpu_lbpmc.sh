#!/bin/bash
# Large-batch step (B=512, k=50) only: kernel trace (per-grid durations), then PMC passes by grid.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-lbpmc}; shift; TUNE="$*"
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u tools/train_large.py 512 10 auto $TUNE > $O/run.log 2>&1 || exit $?
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); python tools/kernel_by_grid.py "$T" > $O/kernel_by_grid.txt; head -24 $O/kernel_by_grid.txt
P=$O/pmc; mkdir -p $P
pass() { local name=$1; shift; timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $P/$name -o run -- python -u tools/train_large.py 512 4 auto $TUNE > $P/$name.log 2>&1; echo "pass $name rc=$?"; }
pass fetch FETCH_SIZE && pass write WRITE_SIZE GRBM_GUI_ACTIVE && \
pass sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES && \
pass sq2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_VALU_MFMA_BUSY_CYCLES && \
pass tcc TCC_HIT_sum TCC_MISS_sum
python tools/pmc_by_grid.py $P "" --json $O/pmc_by_grid.json > $O/pmc_by_grid.txt; echo summary rc=$?
