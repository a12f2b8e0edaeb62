#!/bin/bash
# Write-through hand-off of the combined launch (tcu_kernel): GPU suite on the
# tree, the tcu trace of a write-through trace build, then bench A/B against
# the fence form (libnowt: -DIWAE_TCU_WT=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06r}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
IWAE_HIP_LIB=tools/dbgx/libtcutr2.so timeout -k 10 200 python -u tools/tcu_trace.py 20 > $O/tcu_trace_wt.txt 2>&1 || exit $?
grep -v amdgpu.ids $O/tcu_trace_wt.txt
REPS=3 EXTRA="--no-nll --no-large-batch" bash tools/gpu_benchab.sh ${1:-r06r}/ab tools/dbgx/libnowt.so
