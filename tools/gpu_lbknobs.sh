#!/bin/bash
# B=512 step (tools/train_large.py, fit loop): knob sets given as arguments
# ("knob=v knob=v" each), alternating with the defaults, twice.
#   bash tools/gpu_lbknobs.sh <tag> "tc_img=0" "tc_img=0 tc_imgbwd=0" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-lbknobs}; shift
mkdir -p $O
for rep in 1 2; do
  for t in "" "$@"; do
    timeout -k 10 120 python -u tools/train_large.py 512 40 auto $t 2>/dev/null | sed "s|^|[$t] |" | tee -a $O/lb.txt || exit $?
  done
done
