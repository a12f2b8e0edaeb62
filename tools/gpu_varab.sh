#!/bin/bash
# Variant libraries against the in-tree one: the ring parity tests on each
# variant, then k=5000 NLL images/s and the B=512 step, alternating twice.
#   bash tools/gpu_varab.sh <tag> lib1.so [lib2.so ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-varab}; shift
mkdir -p $O
for lib in "$@"; do
  IWAE_HIP_LIB=$lib timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "${VAR_TESTS:-nll or ring or nring}" > $O/pytest_$(basename $lib).log 2>&1 || { tail -30 $O/pytest_$(basename $lib).log; exit 1; }
  echo "$lib: $(tail -1 $O/pytest_$(basename $lib).log)"
done
for rep in 1 2; do
  for lib in "" "$@"; do
    if [ -n "$lib" ]; then export IWAE_HIP_LIB=$lib; else unset IWAE_HIP_LIB; fi
    timeout -k 10 120 python -u tools/nll_time.py ${NLL_N:-4000} "${lib:-in-tree}" | tee -a $O/nll.txt || exit $?
    timeout -k 10 200 python -u tools/train_large.py 512 40 > $O/large_${rep}_$(basename ${lib:-base}).txt 2>&1 || exit $?
    echo "${lib:-in-tree} large: $(grep -i 'ms' $O/large_${rep}_$(basename ${lib:-base}).txt | tail -1)"
  done
done
