#!/bin/bash
# Per-step time inside short (20-step) vs long (200-step) train_steps calls:
# wall clock without the profiler, then a kernel trace and its per-step spans.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06w; mkdir -p $O
timeout -k 10 120 python -u tools/steps_warm.py run > $O/run.txt 2>&1 || { cat $O/run.txt; exit 1; }
cat $O/run.txt
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python -u tools/steps_warm.py trace > $O/trace_run.txt 2>&1 || { tail $O/trace_run.txt; exit 1; }
P=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/steps_warm.py analyze "$P" > $O/spans.txt 2>&1; cat $O/spans.txt
rm -rf $O/prof
