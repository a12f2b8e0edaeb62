#!/bin/bash
# A/B of library tuning knobs (include/iwae.h enum iwae_knob) on the bench's train legs:
#   TUNES="default upd=0 tc_bound=0,tc_xcd=0" bash tools/ab_tune.sh
# (each word one run; knobs of one run separated by commas; "default" = none)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
i=0
for e in ${TUNES}; do
  i=$((i+1))
  args=""
  if [ "$e" != "default" ]; then for kv in $(echo "$e" | tr ',' ' '); do args="$args --tune $kv"; done; fi
  timeout -k 10 150 python -u bench.py --steps 300 --warmup 20 --no-cpu ${NONLL---no-nll} ${EXTRA:-} $args \
    > gpurun_out/ab/r$i.json 2> gpurun_out/ab/r$i.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/ab/r$i.json').read().strip().splitlines()[-1]); lb=d.get('large_batch') or {}; print('$e', d['ms_per_step'], d['configs0_train']['ms_per_step'] if d.get('configs0_train') else None, lb.get('ms_per_step'), 'nll', (d.get('nll') or {}).get('value'), {n[:14]: v['avg_us'] for n, v in d['roofline']['kernels'].items()})"
done
