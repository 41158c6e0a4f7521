#!/bin/bash
# BLAKE2b lane form: digest GPU tests, then digest timings: quads only, the fused kernel (lanes
# beside quads, RC_B2_LANE_ONLY=0) and the default (the lane kernel when every chunk fits a lane).
set -o pipefail
mkdir -p gpurun_out/lanes
export PYTHONPATH=$PWD/tests:$PWD
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_digest_lanes.py tests/test_gpu_digest.py tests/test_gpu_incremental.py \
    tests/test_gpu_pipeline.py tests/test_gpu_gcm.py > gpurun_out/lanes/pytest.log 2>&1 || { tail -30 gpurun_out/lanes/pytest.log; exit 1; }
tail -3 gpurun_out/lanes/pytest.log
for cfg in "65536 1 2000 80000" "16384 1 2000 80000" "8192 1 2000 80000" "1024 64 128000 5120000"; do
  for mode in quads fused default; do
    unset RC_B2_LANE_MAX RC_B2_LANE_ONLY
    [ $mode = quads ] && export RC_B2_LANE_MAX=0
    [ $mode = fused ] && export RC_B2_LANE_ONLY=0
    echo -n "$mode "
    timeout -k 10 180 python -u scripts/digest_probe.py $cfg || exit 1
  done
done 2>&1 | tee gpurun_out/lanes/probe.log
