#!/bin/bash
# The first encoder layer's pair launch (knob sm_pair: 0 two launches, 1 exact
# f32 pair, 2 bf16x3 l2 pair): equality tests, then an A/B on the bench's train legs
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/${TAG:-r05p}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_edges.py -k "first_encoder_layer" > gpurun_out/${TAG:-r05p}/pytest.log 2>&1 || { tail -30 gpurun_out/${TAG:-r05p}/pytest.log; exit 1; }
tail -3 gpurun_out/${TAG:-r05p}/pytest.log
TUNES="${TUNES:-sm_pair=0 sm_pair=1 sm_pair=2 sm_pair=0 sm_pair=1 sm_pair=2}" timeout -k 10 600 bash tools/ab_tune.sh
