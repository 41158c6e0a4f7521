#!/bin/bash
# round 4: static-schedule launches pipeline now -- overlap / harness parity, the harness line,
# and 3 (iii) in sequence vs pipelined on one allocation
mkdir -p gpurun_out/r04c
timeout -k 10 600 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_harness.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04c/pytest.log 2>&1 || { tail -30 gpurun_out/r04c/pytest.log; exit 1; }
tail -2 gpurun_out/r04c/pytest.log
timeout -k 10 200 python -u bench.py --config harness --steps 20 --warmup 3 > gpurun_out/r04c/bench_harness.log 2>&1 || exit 2
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"pipelined_steps": [0-9]*\|"parity_sha256": [a-z]*\|"kernel_ms": [0-9.]*' gpurun_out/r04c/bench_harness.log
RC_PIPE_ALL=1 AB_STEPS=6 timeout -k 10 300 python -u scripts/overlap_ab.py 3iii 3 seq p32 > gpurun_out/r04c/ab_3iii.log 2>&1 || exit 3
tail -1 gpurun_out/r04c/ab_3iii.log
