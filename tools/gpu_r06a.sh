#!/bin/bash
# Round-6 first check: GPU suite, smoke, default bench line, then one PMC pass
# of instruction-cache counters over the k=5000 NLL leg (2000 images).
#   bash tools/gpu_r06a.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r06a}; O=gpurun_out/$T
mkdir -p $O
bash tools/gpu_round.sh $T || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES \
  --output-format csv -d $O/icache_nll -o run -- python -u tools/nll_time.py 2000 > $O/icache_nll.log 2>&1; echo "icache pass rc=$?"
echo done
