#!/bin/bash
# B=512 step + dw_kernel duration per knob set (no tests):  bash tools/gpu_dwa.sh <tag> "knob=v ..." ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-dwa}; shift
mkdir -p $O
n=0
for cfg in "$@"; do
  T=""; for kv in $cfg; do [ "$kv" != "base" ] && T="$T $kv"; done
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/prof$n -o run -- python -u tools/train_large.py 512 8 auto $T > $O/prof$n.log 2>&1 || exit $?
  F=$(find $O/prof$n -name "*kernel_trace.csv" | head -1)
  echo "[$cfg] $(tail -1 $O/prof$n.log | cut -c1-60)  $(python tools/kernel_by_grid.py "$F" | head -1 | cut -c1-40,70-)"
  n=$((n+1))
done
