#!/bin/bash
# One gpurun call: GPU tests, smoke, the default bench line.
#   bash tools/gpu_round.sh <tag>    (outputs under gpurun_out/<tag>)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-chk}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -2 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.jsonl 2> $O/bench.err || exit $?
tail -1 $O/bench.jsonl
