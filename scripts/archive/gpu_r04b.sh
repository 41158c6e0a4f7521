#!/bin/bash
# round 4 probes: digest overlap with shared vs own hardware queues (HIP's default 4 queues),
# chain-step stamps (diagnostic build) on a harness-sized single stream and on config 2, and the
# harness's tile schedule / pipelining on one allocation
mkdir -p gpurun_out/r04b
# timeout -k 10 300 python -u scripts/digest_overlap_probe.py --queues torch > gpurun_out/r04b/digest_torch.log 2>&1 || exit 1
# timeout -k 10 300 python -u scripts/digest_overlap_probe.py --queues own > gpurun_out/r04b/digest_own.log 2>&1 || exit 1
timeout -k 10 120 python -u scripts/diag_stamps.py 1 4883 > gpurun_out/r04b/stamps_harness.log 2>&1 || exit 1
timeout -k 10 120 python -u scripts/diag_stamps.py 1024 64 > gpurun_out/r04b/stamps_c2.log 2>&1 || exit 1
RC_PIPE_ALL=1 RC_TILE_DYN_MIN=0 AB_STEPS=10 timeout -k 10 300 python -u scripts/overlap_ab.py harness 4 \
    seq@1000:12 seq@100:12 seq@250:32 seq@500:48 p32@1000:12 p32@100:12 p32@250:32 p32@500:48 p32@0:64 \
    > gpurun_out/r04b/harness_sched.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04b/htrace -o run -- python3 bench.py --config harness --steps 5 --warmup 2 --cpu-streams 0 > gpurun_out/r04b/htrace.log 2>&1 || exit 2
python3 scripts/kstats.py gpurun_out/r04b/htrace/run_kernel_stats.csv > gpurun_out/r04b/htrace_stats.txt
cat gpurun_out/r04b/*.log gpurun_out/r04b/*.txt | grep -v progress | tail -90
