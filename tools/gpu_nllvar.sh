#!/bin/bash
# k=5000 NLL images/s: the in-tree library against variant builds (paths as
# arguments), alternating twice; no tests (timing builds).  bash tools/gpu_nllvar.sh <tag> [lib.so ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-nllvar}; shift
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 120 python -u tools/nll_time.py ${NLL_N:-12000} base 2>/dev/null | tee -a $O/nll.txt || exit $?
  for lib in "$@"; do
    IWAE_HIP_LIB=$lib timeout -k 10 120 python -u tools/nll_time.py ${NLL_N:-12000} $lib 2>/dev/null | tee -a $O/nll.txt || exit $?
  done
done
