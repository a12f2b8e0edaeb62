#!/bin/bash
# A/B of library knobs on the train-only bench (B=20 step):  bash tools/gpu_ab.sh <tag> "knob=v ..." "knob=v" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-ab}; shift
mkdir -p $O
for rep in 1 2; do
for cfg in "$@"; do
  T=""; for kv in $cfg; do [ "$kv" != "base" ] && T="$T --tune $kv"; done
  timeout -k 10 200 python -u bench.py --no-cpu --no-nll --no-stats --no-c0 $T > $O/ab.jsonl 2> $O/ab.err || exit $?
  python -c "import json,sys;d=json.loads(open('$O/ab.jsonl').read().splitlines()[-1]);print('$cfg', d['ms_per_step'], d['train_step_calls']['ms_per_step'], d['large_batch']['ms_per_step'])" | tee -a $O/ab.txt
done
done
