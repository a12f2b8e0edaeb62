#!/bin/bash
# GPU suite on the tree (GBWD0 recomputes h1 from eps), then the B=512 step's
# kernels against the previous engine (libprevh: h1 loaded), and the bench's
# train legs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r06i}; O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_libab2.sh $T/lb "tc_kernel|gemm_kernel" tools/dbgx/libprevh.so || exit 1
REPS=2 EXTRA="--no-nll" bash tools/gpu_benchab.sh $T/ab tools/dbgx/libprevh.so
