#!/bin/bash
# B=512 train step (tools/train_large.py): the in-tree library against variant
# builds (paths as arguments), alternating twice.   bash tools/gpu_lbvar.sh <tag> [lib.so ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-lbvar}; shift
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 120 python -u tools/train_large.py 512 40 auto 2>/dev/null | sed "s|^|base |" | tee -a $O/lb.txt || exit $?
  for lib in "$@"; do
    IWAE_HIP_LIB=$lib timeout -k 10 120 python -u tools/train_large.py 512 40 auto 2>/dev/null | sed "s|^|$lib |" | tee -a $O/lb.txt || exit $?
  done
done
