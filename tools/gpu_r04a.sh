set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 200 python -u tools/step_overhead.py > $O/step_overhead.txt 2>&1 || exit $?
cat $O/step_overhead.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
  python -u bench.py --steps 200 --warmup 20 --no-cpu --no-nll --no-large-batch --no-c0 --no-stats > $O/bench.log 2>&1 || exit $?
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/step_gaps.py "$T" > $O/step_gaps.txt; cat $O/step_gaps.txt
