#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
OUT="${PROF_OUT:-gpurun_out/prof}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python -u bench.py --steps "${STEPS:-50}" --warmup 5 --no-cpu ${BENCH_ARGS:-} > gpurun_out/prof_bench.log 2>&1
rc=$?
tail -2 gpurun_out/prof_bench.log
find "$OUT" -name "*stats*" | head
exit $rc
