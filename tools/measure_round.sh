#!/bin/bash
# Round measurement on the GPU box: default bench line, rocprofv3 kernel-trace +
# stats of the same command, PMC passes (train step only) -> the per-launch HBM
# traffic records bench.py reports as roofline.traffic.
#   bash tools/measure_round.sh <tag>      (outputs under gpurun_out/round)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/round
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.jsonl 2> $O/bench.err || exit $?
tail -1 $O/bench.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- \
  python -u bench.py > $O/bench_prof.jsonl 2> $O/bench_prof.err || exit $?
PMC_OUT=$O/pmc bash tools/pmc_passes.sh python -u bench.py --steps 20 --warmup 5 --no-nll --no-cpu --no-c0 \
  --no-large-batch || exit $?
python tools/pmc_to_json.py $O/pmc "tc_kernel<" $O/pmc_traffic.json "tc_kernel forward (train engine, bf16x3)" rank:0 &&
python tools/pmc_to_json.py $O/pmc "tc_kernel<" $O/pmc_traffic.json "tc_kernel backward (train engine, bf16x3)" rank:1 &&
python tools/pmc_to_json.py $O/pmc "upd_kernel" $O/pmc_traffic.json "upd_kernel (weight gradients + Adam + FX copies, bf16x3)" max &&
python tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt &&
PROF_OUT=$O/pstep bash tools/prof_step.sh > /dev/null
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); python tools/kernel_by_grid.py "$T" > $O/kernel_by_grid.txt
