#!/bin/bash
# B=20 kernel durations (rocprofv3 --kernel-trace of tools/steps_b20.py) for the
# in-tree library and each variant library given: bash tools/gpu_sptrace.sh <tag> [lib.so ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-sptrace}; shift
mkdir -p $O
n=0
for lib in "" "$@"; do
  if [ -n "$lib" ]; then export IWAE_HIP_LIB=$lib; else unset IWAE_HIP_LIB; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/p$n -o run -- \
    python -u tools/steps_b20.py 64 ${SP_TUNE:-} > $O/p$n.log 2>&1 || exit $?
  F=$(find $O/p$n -name "*kernel_trace.csv" | head -1)
  echo "== ${lib:-in-tree}"; python tools/kernel_by_grid.py "$F" | head -12
  n=$((n+1))
done
