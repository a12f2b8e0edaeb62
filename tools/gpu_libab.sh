#!/bin/bash
# B=512 step and per-kernel durations: the in-tree library against a variant
# build (path), alternating twice, each under rocprofv3 --kernel-trace.
#   bash tools/gpu_libab.sh <tag> <lib.so> [kernel name filter]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-libab}; LIB=$2; K=${3:-dw_kernel}
mkdir -p $O
n=0
for rep in 1 2; do
  for lib in "" "$LIB"; do
    if [ -n "$lib" ]; then export IWAE_HIP_LIB=$lib; else unset IWAE_HIP_LIB; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/p$n -o run -- \
      python -u tools/train_large.py 512 16 auto > $O/p$n.log 2>&1 || exit $?
    F=$(find $O/p$n -name "*kernel_trace.csv" | head -1)
    echo "[${lib:-in-tree}] $(grep -o 'B=512.*ms/step' $O/p$n.log) | $(python tools/kernel_by_grid.py "$F" | grep "$K" | sed 's/  */ /g' | cut -c1-100)"
    n=$((n+1))
  done
done
