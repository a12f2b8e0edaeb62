#!/bin/bash
# B=512 step A/B: per knob set, the step time and the per-(kernel, grid) durations (kernel trace)
#   bash tools/gpu_lbab.sh <tag> "knob=v ..." ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-lbab}; shift
mkdir -p $O
n=0
for cfg in "$@"; do
  T=""; for kv in $cfg; do [ "$kv" != "base" ] && T="$T $kv"; done
  timeout -k 10 120 python -u tools/train_large.py 512 20 auto $T > $O/run$n.log 2>&1 || exit $?
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/prof$n -o run -- python -u tools/train_large.py 512 8 auto $T > $O/prof$n.log 2>&1 || exit $?
  F=$(find $O/prof$n -name "*kernel_trace.csv" | head -1)
  echo "== [$cfg] $(grep ms/step $O/run$n.log)"
  python tools/kernel_by_grid.py "$F" > $O/kbg$n.txt; awk '$0 ~ /avg/ {print}' $O/kbg$n.txt | head -12 | cut -c1-45,70-120
  n=$((n+1))
done
