#!/bin/bash
# GPU-box check: parity tests, smoke, short bench. Stops at the first step that
# faults, aborts or times out (exit codes other than 0/1 from pytest).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS="${STEPS:-200}"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
src=$?
cat gpurun_out/smoke.log | tail -3
if [ $src -ne 0 ] && [ $src -ne 1 ]; then echo "smoke rc=$src: stopping"; exit $src; fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 400 python -u bench.py --steps "$STEPS" --warmup 20 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
  brc=$?
  tail -3 gpurun_out/bench.log
  if [ $brc -ne 0 ]; then echo "bench rc=$brc"; exit $brc; fi
fi
echo "pytest rc=$rc smoke rc=$src"
