#!/bin/bash
# kernel trace of the large-batch leg (B=512, k=50) -> per-grid kernel durations
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-lbprof}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python -u bench.py --steps 5 --warmup 2 --no-nll --no-cpu --no-c0 --no-stats --large-batch-steps 10 > $O/bench.log 2>&1 || exit $?
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); python tools/kernel_by_grid.py "$T" > $O/kernel_by_grid.txt; head -30 $O/kernel_by_grid.txt
