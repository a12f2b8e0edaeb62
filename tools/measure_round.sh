#!/bin/bash
# Round measurement on the GPU box (outputs under gpurun_out/<tag>):
#   the default bench line and one with the driver's arguments (--steps 20
#   --warmup 5), rocprofv3 --kernel-trace --stats of the bench, PMC passes of
#   the B = 20 step (separate passes, kernel trace only) -> the per-launch HBM
#   traffic records bench.py reports as roofline.traffic, the step timeline.
#   bash tools/measure_round.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-round}
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench.jsonl 2> $O/bench.err || exit $?
tail -c 400 $O/bench.jsonl
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_driver.jsonl 2> $O/bench_driver.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- \
  python -u bench.py --no-cpu > $O/bench_prof.jsonl 2> $O/bench_prof.err || exit $?
PMC_OUT=$O/pmc bash tools/pmc_passes.sh python -u bench.py --steps 20 --warmup 5 --no-nll --no-cpu --no-c0 \
  --no-large-batch --no-stats || exit $?
J=$O/pmc_traffic.json
python tools/pmc_to_json.py $O/pmc "tc_kernel<" $J "tc_kernel forward (train engine, bf16x3)" rank:0 &&
python tools/pmc_to_json.py $O/pmc "tc_kernel<" $J "tc_kernel backward (train engine, bf16x3)" rank:1 &&
python tools/pmc_to_json.py $O/pmc "upd_kernel" $J "upd_kernel (weight gradients + Adam + FX copies, bf16x3)" max &&
python tools/pmc_to_json.py $O/pmc "tcu_kernel" $J "tcu_kernel (job I' + weight gradients + Adam + FX copies, one launch)" max &&
python tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt &&
PROF_OUT=$O/pstep NK=7 FIRST="smallm_kernel<false, 2, 1>@52" bash tools/prof_step.sh > /dev/null
T=$(find $O/prof -name "*kernel_trace.csv" | head -1); python tools/kernel_by_grid.py "$T" > $O/kernel_by_grid.txt
echo measure done
