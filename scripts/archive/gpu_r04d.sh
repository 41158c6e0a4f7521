#!/bin/bash
# round 4: the snapshot producer end to end (8 GiB in 128 files; run() vs the zero-copy
# stream()), and a two-rank rehearsal of the N-GPU line on the one-GPU lease (--share-gpus):
# every rank checks its own shard against tests/golden/ranks.json
mkdir -p gpurun_out/r04d
export TMPDIR=/tmp
timeout -k 10 420 python -u scripts/producer_probe.py 8192 128 > gpurun_out/r04d/producer_8g.log 2>&1
echo "producer rc=$?"; grep '^{' gpurun_out/r04d/producer_8g.log | cut -c1-330
timeout -k 10 300 python -u bench.py --gpus 2 --share-gpus --steps 10 --warmup 2 > gpurun_out/r04d/ranks2.log 2>&1 || { echo "ranks2 failed"; tail -20 gpurun_out/r04d/ranks2.log; exit 2; }
grep -o '"value": [0-9.]*\|"parity_sha256": [a-z]*\|"parity_scope": "[^"]*"\|"cores": [0-9]*' gpurun_out/r04d/ranks2.log
