#!/bin/bash
# Large-batch (configs[4] per-GPU share) A/B of library tuning knobs:
#   TUNES="default wide_rows=100000000 upd_slab_wg=768" bash tools/lb_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lb
i=0
for e in ${TUNES}; do
  i=$((i+1))
  args=""
  if [ "$e" != "default" ]; then for kv in $(echo "$e" | tr ',' ' '); do args="$args --tune $kv"; done; fi
  timeout -k 10 150 python -u bench.py --steps 30 --warmup 5 --no-cpu --no-nll --no-c0 $args \
    > gpurun_out/lb/b$i.json 2> gpurun_out/lb/b$i.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/lb/b$i.json').read().strip().splitlines()[-1]); print('$e', d['ms_per_step'], d['large_batch']['ms_per_step'])"
done
