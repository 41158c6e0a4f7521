#!/bin/bash
# round 4, first GPU pass: the whole GPU suite, then the default bench line
mkdir -p gpurun_out/r04a
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04a/pytest.log 2>&1
echo "pytest rc=$?"
tail -3 gpurun_out/r04a/pytest.log
timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r04a/bench.log 2>&1
echo "bench rc=$?"
tail -c 2500 gpurun_out/r04a/bench.log
