#!/bin/bash
# Final round-5 records of the tree (outputs under gpurun_out/<tag>): GPU suite,
# smoke, the default bench line and one with the driver's arguments, rocprofv3
# --kernel-trace --stats of the bench, the B = 20 step timeline, and one PMC
# pass of instruction-cache counters over the B = 20 steps (SQ block, 6 of 8).
#   bash tools/gpu_final5.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${1:-r05h}; O=gpurun_out/$T
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
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
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES \
  --output-format csv -d $O/icache -o run -- python -u tools/steps_b20.py 20 > $O/icache.log 2>&1; echo "icache pass rc=$?"
echo final done
