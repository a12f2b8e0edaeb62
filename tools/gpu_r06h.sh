#!/bin/bash
# Engine op timelines (tc_trace.py on a -DIWAE_TC_TRACE build): B = 512 (the
# image-row jobs I / I') and B = 20.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-r06h}; mkdir -p $O
IWAE_HIP_LIB=tools/dbgx/libtctr.so timeout -k 10 120 python -u tools/tc_trace.py 512 > $O/tc_trace_512.txt 2>&1 || { tail $O/tc_trace_512.txt; exit 1; }
IWAE_HIP_LIB=tools/dbgx/libtctr.so timeout -k 10 120 python -u tools/tc_trace.py 20 > $O/tc_trace_20.txt 2>&1 || { tail $O/tc_trace_20.txt; exit 1; }
cat $O/tc_trace_512.txt | head -60
echo ====
cat $O/tc_trace_20.txt | head -60
