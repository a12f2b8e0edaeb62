set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
IWAE_HIP_LIB=tools/_dbg/libiwae_tctrace.so timeout -k 10 120 python -u tools/tc_trace.py 512 50 > gpurun_out/tctrace512.txt 2>&1 || exit $?
head -12 gpurun_out/tctrace512.txt
