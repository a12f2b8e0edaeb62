#!/bin/bash
# GPU suite on the tree, then A/B of the in-tree library against: the combined
# launch without its SHORT instantiation (libnoshort), and nre_kernel with the
# round-5 E1 staging strides (libnreold): bench train legs + per-kernel trace.
#   bash tools/gpu_r06f.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r06f}; O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
REPS=3 EXTRA="--no-nll --no-large-batch" bash tools/gpu_benchab.sh $T/short tools/dbgx/libnoshort.so || exit 1
bash tools/gpu_libab2.sh $T/lb "nre_kernel|gemm_kernel|tc_kernel" tools/dbgx/libnreold.so tools/dbgx/libfs8.so tools/dbgx/libfs4.so
