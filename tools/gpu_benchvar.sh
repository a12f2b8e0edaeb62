#!/bin/bash
# Train-step legs of bench.py (B=20 headline + B=512) for the in-tree library
# against variant builds (paths as arguments), alternating twice.
#   bash tools/gpu_benchvar.sh <tag> [lib.so ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-benchvar}; shift
mkdir -p $O
for rep in 1 2; do
  for lib in base "$@"; do
    if [ "$lib" = base ]; then unset IWAE_HIP_LIB; else export IWAE_HIP_LIB=$lib; fi
    timeout -k 10 200 python -u bench.py --no-cpu --no-nll --no-stats --no-c0 > $O/b.jsonl 2> $O/b.err || exit $?
    python -c "import json;d=json.loads(open('$O/b.jsonl').read().splitlines()[-1]);print('$lib', d['ms_per_step'], d['train_step_calls']['ms_per_step'], d['large_batch']['ms_per_step'])" | tee -a $O/ab.txt
  done
done
