set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_state.py tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt8.log 2>&1; rc=$?
tail -4 gpurun_out/pt8.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
TUNES="default dw_wide=0 wide_rows=100000000" bash tools/lb_ab.sh || exit $?
IWAE_HIP_LIB=tools/_dbg/libiwae_tctrace.so timeout -k 10 120 python -u tools/tc_trace.py 512 50 > gpurun_out/tctrace512b.txt 2>&1 || exit $?
head -7 gpurun_out/tctrace512b.txt
