#!/bin/bash
# GPU suite on the tree (nre_kernel's E1 staging strides), nre_kernel LDS
# counters, dw_kernel variants (fragment prefetch depth, no SLP) per kernel,
# and the engine files without the SLP vectorizer on the bench legs.
#   bash tools/gpu_r06d.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r06d}; O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES \
  --output-format csv -d $O/pmc_nre -o run -- python -u tools/train_large.py 512 10 > $O/pmc_nre.log 2>&1 || { echo "pmc failed"; exit 1; }
python tools/pmc_kernel.py $(find $O/pmc_nre -name "*counter_collection.csv" | head -1) nre_kernel | tee $O/pmc_nre.txt
bash tools/gpu_libab2.sh $T/dw "dw_kernel|nre_kernel" tools/dbgx/libdwpf2.so tools/dbgx/libdwpf3.so tools/dbgx/libdwnoslp.so || exit 1
REPS=3 NLL_N=3000 bash tools/gpu_benchab.sh $T/trnoslp tools/dbgx/libtrnoslp.so
