#!/bin/bash
# Traces: ring-kernel unit timeline, train-engine op timeline, the replayed train-step kernel timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-trace}
mkdir -p $O
IWAE_HIP_LIB=tools/_dbg/libiwae_nrtrace.so timeout -k 10 120 python -u tools/nr_trace.py > $O/nr_trace.txt 2>&1 || exit $?
head -3 $O/nr_trace.txt | grep -v amdgpu
IWAE_HIP_LIB=tools/_dbg/libiwae_tctrace.so timeout -k 10 120 python -u tools/tc_trace.py > $O/tc_trace.txt 2>&1 || exit $?
PROF_OUT=$O/pstep NK=7 timeout -k 10 300 bash tools/prof_step.sh > $O/timeline.txt 2>&1 || exit $?
cat $O/timeline.txt | tail -12
