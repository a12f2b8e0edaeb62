#!/bin/bash
# (1) nre_kernel LDS bank conflicts per ablation build (SQ_LDS_BANK_CONFLICT /
# SQ_LDS_IDX_ACTIVE over the B=512 step), (2) the stagger variants against the
# in-tree library (parity + NLL + B=512).
#   bash tools/gpu_r06c.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r06c}; O=gpurun_out/$T
mkdir -p $O
for lib in "" tools/dbgx/libnre1.so tools/dbgx/libnre2.so tools/dbgx/libnre4.so tools/dbgx/libnre8.so tools/dbgx/libnre16.so; do
  if [ -n "$lib" ]; then export IWAE_HIP_LIB=$lib; else unset IWAE_HIP_LIB; fi
  n=$(basename ${lib:-base.so} .so)
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES \
    --output-format csv -d $O/pmc_$n -o run -- python -u tools/train_large.py 512 10 > $O/pmc_$n.log 2>&1 || { echo "pmc $n failed"; tail -5 $O/pmc_$n.log; exit 1; }
  F=$(find $O/pmc_$n -name "*counter_collection.csv" | head -1)
  echo "== $n"; python tools/pmc_kernel.py "$F" nre_kernel | tee $O/pmc_$n.txt
done
unset IWAE_HIP_LIB
bash tools/gpu_varab.sh $T/st tools/dbgx/libst1.so tools/dbgx/libst2.so
# (3) every kernel compiled without the SLP vectorizer (no packed f32 VALU):
# the whole GPU suite on it, then the bench legs against the in-tree library
VAR_TESTS="gpu" REPS=2 NLL_N=4000 bash tools/gpu_benchab.sh $T/noslp tools/dbgx/libnoslp.so
