set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_state.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt6.log 2>&1; rc=$?
tail -4 gpurun_out/pt6.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
TUNES="default ld_align=32 ld_align=32,dw_wide=0" bash tools/lb_ab.sh || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc6/w -o run -- python -u tools/train_large.py 512 5 > gpurun_out/pmc6_w.log 2>&1 || exit $?
python tools/pmc_summary.py gpurun_out/pmc6 | grep -A3 'tc_kernel\|dw_kernel'
