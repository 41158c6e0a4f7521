#!/bin/bash
# round 4 probes: digest overlap with shared vs own hardware queues (HIP's default 4 queues),
# chain-step stamps (diagnostic build) on a harness-sized single stream and on config 2
mkdir -p gpurun_out/r04b
timeout -k 10 300 python -u scripts/digest_overlap_probe.py --queues torch > gpurun_out/r04b/digest_torch.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/digest_overlap_probe.py --queues own > gpurun_out/r04b/digest_own.log 2>&1 || exit 1
timeout -k 10 120 python -u scripts/diag_stamps.py 1 4883 > gpurun_out/r04b/stamps_harness.log 2>&1 || exit 1
timeout -k 10 120 python -u scripts/diag_stamps.py 1024 64 > gpurun_out/r04b/stamps_c2.log 2>&1 || exit 1
cat gpurun_out/r04b/*.log | grep -v progress | tail -60
