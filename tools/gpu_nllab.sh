#!/bin/bash
# NLL parity tests, then k=5000 NLL images/s: the in-tree library against
# variant builds (paths as arguments), alternating twice; plus the B=512 step.
#   bash tools/gpu_nllab.sh <tag> [lib.so ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-nllab}; shift
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "nll or ring or nring or configs or piwae" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
  timeout -k 10 120 python -u tools/nll_time.py ${NLL_N:-4000} base | tee -a $O/nll.txt || exit $?
  for lib in "$@"; do
    IWAE_HIP_LIB=$lib timeout -k 10 120 python -u tools/nll_time.py ${NLL_N:-4000} $lib | tee -a $O/nll.txt || exit $?
  done
done
timeout -k 10 200 python -u tools/train_large.py 512 20 auto > $O/large.txt 2>&1 && tail -3 $O/large.txt
