#!/bin/bash
# Job I''s Gaussian backward in one load round trip (the first sample batch and
# the image's (mu, zs) requested together, 4 samples per thread at one image
# per workgroup): GPU suite on the tree, then bench A/B (B=20, configs[0],
# B=512) against the previous tree (libgb0old).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06t}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
REPS=3 EXTRA="--no-nll" bash tools/gpu_benchab.sh ${1:-r06t}/ab tools/dbgx/libgb0old.so
