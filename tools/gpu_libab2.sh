#!/bin/bash
# B=512 step and per-kernel durations (rocprofv3 --kernel-trace): the in-tree
# library against variant builds, alternating REPS times.
#   bash tools/gpu_libab2.sh <tag> <kernel filter regex> lib1.so [lib2.so ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-libab2}; K=$2; shift 2
mkdir -p $O
n=0
for rep in $(seq 1 ${REPS:-2}); do
  for lib in "" "$@"; do
    if [ -n "$lib" ]; then export IWAE_HIP_LIB=$lib; else unset IWAE_HIP_LIB; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/p$n -o run -- \
      python -u tools/train_large.py 512 16 auto > $O/p$n.log 2>&1 || exit $?
    F=$(find $O/p$n -name "*kernel_trace.csv" | head -1)
    echo "[${lib:-in-tree}] $(grep -o 'B=512.*ms/step' $O/p$n.log)"
    python tools/kernel_by_grid.py "$F" | grep -E "$K" | sed 's/  */ /g' | cut -c1-110
    n=$((n+1))
  done
done
