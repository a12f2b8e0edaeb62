#!/bin/bash
# Round measurement on the GPU box: default bench line, rocprofv3 kernel-trace +
# stats of the same command, PMC passes (train step only) for roofline.traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/round
timeout -k 10 400 python -u bench.py > gpurun_out/round/bench.jsonl 2> gpurun_out/round/bench.err || exit $?
tail -1 gpurun_out/round/bench.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/round/prof -o bench -- \
  python -u bench.py > gpurun_out/round/bench_prof.jsonl 2> gpurun_out/round/bench_prof.err || exit $?
PMC_OUT=gpurun_out/round/pmc bash tools/pmc_passes.sh python -u bench.py --steps 20 --warmup 5 --no-nll --no-cpu
