#!/bin/bash
# rocprofv3 kernel trace of replayed headline steps (tools/steps_b20.py) and the kernel
# timeline of one train step (tools/step_timeline.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT="${PROF_OUT:-gpurun_out/pstep}"
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python -u tools/steps_b20.py 30 > "$OUT/bench.log" 2>&1 || exit $?
T=$(find "$OUT" -name "*kernel_trace.csv" | head -1)
python tools/step_timeline.py "$T" "${NK:-12}" "${FIRST:-smallm_kernel<false>}" | tee "$OUT/timeline.txt"
