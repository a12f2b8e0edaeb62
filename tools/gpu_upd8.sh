#!/bin/bash
# Update-kernel wave count gate: the whole GPU suite, then A/B of upd_waves on the B=20 and B=512 steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-upd8}
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
EXTRA="--no-large-batch --no-c0 --no-stats" TUNES="default upd_waves=8 default upd_waves=8" bash tools/ab_tune.sh || exit $?
TUNES="default upd_waves=8" bash tools/lb_ab.sh
