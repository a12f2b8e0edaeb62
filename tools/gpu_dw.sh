#!/bin/bash
# weight-gradient pass gate: its parity tests, then the B=512 step timing and kernel trace for each tuning
#   bash tools/gpu_dw.sh <tag> "knob=v ..." ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-dw}; shift
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_state.py -x -q --timeout 120 --timeout-method thread -k "dw or slab or wide or piwae" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
n=0
for cfg in "$@"; do
  T=""; for kv in $cfg; do [ "$kv" != "base" ] && T="$T $kv"; done
  timeout -k 10 120 python -u tools/train_large.py 512 20 auto $T 2>&1 | tail -1 | sed "s/^/[$cfg] /"
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/prof$n -o run -- python -u tools/train_large.py 512 6 auto $T > $O/prof$n.log 2>&1 || exit $?
  F=$(find $O/prof$n -name "*kernel_trace.csv" | head -1); python tools/kernel_by_grid.py "$F" > $O/kbg$n.txt; head -3 $O/kbg$n.txt
  n=$((n+1))
done
