#!/bin/bash
# GPU suite on the tree, then the B=512 step with the first encoder layer's
# input GEMM in fewer split-K slabs (libfs8 / libfs4) against the in-tree 13.
#   bash tools/gpu_r06g.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r06g}; O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for lib in tools/dbgx/libfs8.so tools/dbgx/libfs4.so; do
  IWAE_HIP_LIB=$lib timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "512 or large or slab or input_gemm" > $O/pytest_$(basename $lib).log 2>&1 || { tail -30 $O/pytest_$(basename $lib).log; exit 1; }
  echo "$lib: $(tail -1 $O/pytest_$(basename $lib).log)"
done
bash tools/gpu_libab2.sh $T/lb "gemm_kernel|tc_kernel|bound" tools/dbgx/libfs8.so tools/dbgx/libfs4.so
