#!/bin/bash
# BLAKE2b lane form: digest GPU tests, then digest timings with lanes off / default / all.
set -o pipefail
mkdir -p gpurun_out/lanes
export PYTHONPATH=$PWD/tests:$PWD
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_digest_lanes.py tests/test_gpu_digest.py tests/test_gpu_incremental.py \
    tests/test_gpu_pipeline.py tests/test_gpu_gcm.py > gpurun_out/lanes/pytest.log 2>&1 || { tail -30 gpurun_out/lanes/pytest.log; exit 1; }
tail -3 gpurun_out/lanes/pytest.log
for cfg in "65536 1 2000 80000" "1024 64 128000 5120000" "4096 1 2000 80000" "8192 1 2000 80000"; do
  for lm in 0 default; do
    if [ "$lm" = default ]; then unset RC_B2_LANE_MAX; else export RC_B2_LANE_MAX=$lm; fi
    echo -n "lane_max=$lm "
    timeout -k 10 180 python -u scripts/digest_probe.py $cfg || exit 1
  done
done 2>&1 | tee gpurun_out/lanes/probe.log
