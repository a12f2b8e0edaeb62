#!/bin/bash
# Instruction-cache counters of the B = 512 step's kernels (one PMC pass over
# tools/train_large.py 512): which of them miss their 64 KB instruction cache.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06ic; mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
  --output-format csv -d $O/pmc -o run -- python -u tools/train_large.py 512 4 auto > $O/run.log 2>&1; echo "pass rc=$?"
P=$(find $O/pmc -name "*counter_collection.csv" | head -1); [ -n "$P" ] && python tools/pmc_kernel.py "$P" > $O/icache_b512.txt 2>&1; cat $O/icache_b512.txt
rm -rf $O/pmc
