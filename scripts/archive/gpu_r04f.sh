#!/bin/bash
# round 4: BLAKE2b quad G with the message word added first (one dependent add after b):
# config-2 batch digests, previous library vs this one (latency-bound: the 5 MB chains), then
# the digest parity tests
mkdir -p gpurun_out/r04f
for k in 1 2; do
  RC_LIB_PATH=diag/lib_PREVB2.so timeout -k 10 120 python -u scripts/digest_probe.py > gpurun_out/r04f/prev_$k.log 2>&1 || exit 1
  timeout -k 10 120 python -u scripts/digest_probe.py > gpurun_out/r04f/new_$k.log 2>&1 || exit 1
done
grep -h '^{' gpurun_out/r04f/prev_*.log gpurun_out/r04f/new_*.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_digest.py tests/test_gpu_digest_lanes.py tests/test_gpu_incremental.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04f/pytest.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/r04f/pytest.log
