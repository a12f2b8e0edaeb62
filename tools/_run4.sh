set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_schedule.py tests/test_gpu_state.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt4.log 2>&1; rc=$?
tail -8 gpurun_out/pt4.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
TUNES="default dw_wide=0 wide_rows=100000000" bash tools/lb_ab.sh || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lbprof4 -o lb -- python -u tools/train_large.py 512 20 > gpurun_out/lbprof4.log 2>&1 || exit $?
T=$(find gpurun_out/lbprof4 -name "*kernel_trace.csv" | head -1); python tools/kernel_by_grid.py "$T" > gpurun_out/lb4_kernel_by_grid.txt; head -12 gpurun_out/lb4_kernel_by_grid.txt
