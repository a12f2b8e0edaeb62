#!/bin/bash
# Engine op timelines (first workgroup of every job) of B = 20 eager steps on a
# -DIWAE_TC_TRACE build (tools/dbgx/libtctrace.so): where job I' spends its time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r06y; mkdir -p $O
IWAE_HIP_LIB=tools/dbgx/libtctrace.so timeout -k 10 120 python -u tools/tc_trace.py 20 > $O/tc_trace_b20.txt 2>&1 || { tail $O/tc_trace_b20.txt; exit 1; }
cat $O/tc_trace_b20.txt
