#!/bin/bash
# Narrow engine instantiations: job I (B > 32 images) on tc_kernel<1, kTcKindsImgFwd>
# (31 KB of code instead of the 66 KB forward set), and the B = 20 forward launch
# on tc_kernel<1, kTcKindsFwdRows> (63.7 KB: without the folded image-row ops).
# Parity subset, then the bench (B = 20, configs[0], B = 512) alternating:
# in-tree, without the forward-rows set (libnofr), the previous library (libnoif).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06if; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "512 or configs or image_row or engine" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
REPS=3 EXTRA="--no-nll" bash tools/gpu_benchab.sh r06if_ab tools/dbgx/libnofr.so tools/dbgx/libnoif.so
