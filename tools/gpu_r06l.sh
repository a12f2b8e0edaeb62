#!/bin/bash
# GPU suite on the tree (NLL: first encoder layer once per group of ~16 K
# images), then the NLL leg (10 k images) against the previous host code.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r06l}; O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
REPS=3 NLL_N=10000 EXTRA="--no-large-batch --no-c0" bash tools/gpu_benchab.sh $T/ab tools/dbgx/libprevnll.so
