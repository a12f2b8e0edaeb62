#!/bin/bash
# Instruction-cache counters of the B = 20 step's kernels on the final tree
# (the -Os train engine), one PMC pass over tools/steps_b20.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06ic20; mkdir -p $O
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES \
  --output-format csv -d $O/pmc -o run -- python -u tools/steps_b20.py 20 > $O/run.log 2>&1; echo "pass rc=$?"
P=$(find $O/pmc -name "*counter_collection.csv" | head -1); [ -n "$P" ] && python tools/pmc_kernel.py "$P" iwae > $O/icache_b20.txt 2>&1; cat $O/icache_b20.txt
rm -rf $O/pmc
