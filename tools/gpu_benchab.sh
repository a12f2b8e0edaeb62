#!/bin/bash
# Whole-bench A/B of variant libraries against the in-tree one (B=20 headline,
# configs[0], k=5000 NLL, B=512), alternating REPS times on one box; optional
# parity subset on each variant first (VAR_TESTS, pytest -k expression).
#   bash tools/gpu_benchab.sh <tag> lib1.so [lib2.so ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-benchab}; shift
mkdir -p $O
if [ -n "${VAR_TESTS:-}" ]; then
  for lib in "$@"; do
    IWAE_HIP_LIB=$lib timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      -k "$VAR_TESTS" > $O/pytest_$(basename $lib).log 2>&1 || { tail -30 $O/pytest_$(basename $lib).log; exit 1; }
    echo "$lib: $(tail -1 $O/pytest_$(basename $lib).log)"
  done
fi
i=0
for rep in $(seq 1 ${REPS:-2}); do
  for lib in "" "$@"; do
    i=$((i+1))
    if [ -n "$lib" ]; then export IWAE_HIP_LIB=$lib; else unset IWAE_HIP_LIB; fi
    timeout -k 10 200 python -u bench.py --steps 300 --warmup 20 --no-cpu --no-stats --nll-images ${NLL_N:-6000} ${EXTRA:-} \
      > $O/r$i.json 2> $O/r$i.err || { tail -5 $O/r$i.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/r$i.json').read().strip().splitlines()[-1]); lb=d.get('large_batch') or {}; print('${lib:-in-tree}', 'b20', d['ms_per_step'], 'c0', (d.get('configs0_train') or {}).get('ms_per_step'), 'nll', (d.get('nll') or {}).get('value'), 'b512', lb.get('ms_per_step'))" | tee -a $O/summary.txt
  done
done
