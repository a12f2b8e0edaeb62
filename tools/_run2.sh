set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_schedule.py tests/test_gpu_state.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pt2.log 2>&1; rc=$?
tail -15 gpurun_out/pt2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
TUNES="default wide_rows=100000000" bash tools/lb_ab.sh
