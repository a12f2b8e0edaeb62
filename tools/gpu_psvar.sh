#!/bin/bash
# Priority-split experiment (IWAE_PS_* builds): NLL, B=512 step and B=20 step
# for a base debug build against variants, alternating twice.
#   bash tools/gpu_psvar.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-psvar}
mkdir -p $O
for rep in 1 2; do
  for v in base NR; do
    IWAE_HIP_LIB=dbgx/libps_$v.so timeout -k 10 120 python -u tools/nll_time.py 12000 $v 2>/dev/null | tee -a $O/nll.txt || exit $?
  done
  for v in base NR DW NRBE; do
    echo -n "$v " | tee -a $O/lb.txt
    IWAE_HIP_LIB=dbgx/libps_$v.so timeout -k 10 120 python -u tools/train_large.py 512 40 2>/dev/null | tee -a $O/lb.txt || exit $?
  done
  for v in base TC; do
    IWAE_HIP_LIB=dbgx/libps_$v.so timeout -k 10 200 python -u bench.py --no-cpu --no-nll --no-stats --no-c0 --no-large-batch > $O/b.jsonl 2> $O/b.err || exit $?
    python -c "import json;d=json.loads(open('$O/b.jsonl').read().splitlines()[-1]);print('$v', d['ms_per_step'], d['train_step_calls']['ms_per_step'])" | tee -a $O/b20.txt
  done
done
