#!/bin/bash
# GPU suite on the tree (tcu_kernel without the multi-group update path), the
# suite on the engine variant (one unit loop, two epilogue sites + no SLP),
# then the bench's train legs: in-tree vs variants, alternating 3 times.
#   bash tools/gpu_r06e.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r06e}; O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
VAR_TESTS="gpu" REPS=3 EXTRA="--no-nll" bash tools/gpu_benchab.sh $T/ab tools/dbgx/libepi2.so tools/dbgx/libepi2ns.so tools/dbgx/libtrnoslp.so
