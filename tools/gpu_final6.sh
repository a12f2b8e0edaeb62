#!/bin/bash
# Final round-6 records of the tree (outputs under gpurun_out/<tag>), in two
# gpurun calls:
#   part a: GPU suite, smoke, the default bench line and one with the driver's
#           arguments, rocprofv3 --kernel-trace --stats of the bench, the B = 20
#           step timeline;
#   part b: the B = 20 step's PMC passes (separate passes, kernel trace only) ->
#           the per-launch HBM traffic record bench.py reports as
#           roofline.traffic, then the B = 512 step's kernel trace + PMC passes
#           (tools/gpu_lbpmc.sh) -> the large-batch kernel record.
#   bash tools/gpu_final6.sh <tag> a|b
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r06}; O=gpurun_out/$T
mkdir -p $O
if [ "${2:-a}" = a ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
  tail -1 $O/smoke.log
  timeout -k 10 400 python -u bench.py > $O/bench.jsonl 2> $O/bench.err || exit $?
  tail -c 300 $O/bench.jsonl; echo
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_driver_args.jsonl 2> $O/bench_driver.err || exit $?
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- \
    python -u bench.py --no-cpu > $O/bench_prof.jsonl 2> $O/bench_prof.err || exit $?
  P=$(find $O/prof -name "*kernel_trace.csv" | head -1); python tools/kernel_by_grid.py "$P" > $O/kernel_by_grid.txt
  PROF_OUT=$O/pstep NK=7 FIRST="smallm_kernel<false, 2, 1>@52" bash tools/prof_step.sh > /dev/null || exit $?
else
  PMC_OUT=$O/pmc bash tools/pmc_passes.sh python -u bench.py --steps 20 --warmup 5 --no-nll --no-cpu --no-c0 \
    --no-large-batch --no-stats || exit $?
  J=$O/pmc_traffic.json
  python tools/pmc_to_json.py $O/pmc "tc_kernel<" $J "tc_kernel forward (train engine, bf16x3)" rank:0 &&
  python tools/pmc_to_json.py $O/pmc "tc_kernel<" $J "tc_kernel backward (train engine, bf16x3)" rank:1 &&
  python tools/pmc_to_json.py $O/pmc "upd_kernel" $J "upd_kernel (weight gradients + Adam + FX copies, bf16x3)" max &&
  python tools/pmc_to_json.py $O/pmc "tcu_kernel" $J "tcu_kernel (job I' + weight gradients + Adam + FX copies, one launch)" max &&
  python tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt || exit $?
  bash tools/gpu_lbpmc.sh $T/lb > $O/lbpmc.log 2>&1 || { tail -5 $O/lbpmc.log; exit 1; }
  tail -3 $O/lbpmc.log
fi
echo final $2 done
