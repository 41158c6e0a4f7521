#!/bin/bash
# round 4: the guided tail (RC_TILE_GUIDED) against the plain 12-tile units on one allocation per
# config, and the new build (guided off) against the previous library (diag/lib_PREV.so: the
# tile kernel before the guided fields) for the SGPR-spill question
mkdir -p gpurun_out/r04e
timeout -k 10 240 python -u scripts/tile_sched_ab.py 2 8 100:12 100:12:G > gpurun_out/r04e/ab2.log 2>&1 || exit 1
tail -1 gpurun_out/r04e/ab2.log
timeout -k 10 200 python -u scripts/tile_sched_ab.py 3iii 6 100:12 100:12:G > gpurun_out/r04e/ab3iii.log 2>&1 || exit 1
tail -1 gpurun_out/r04e/ab3iii.log
timeout -k 10 300 python -u scripts/tile_sched_ab.py 4 4 100:12 100:12:G > gpurun_out/r04e/ab4.log 2>&1 || exit 1
tail -1 gpurun_out/r04e/ab4.log
timeout -k 10 240 python -u scripts/lib_ab.py 2 8 diag/lib_PREV.so replicat_amd/libreplicat_chunker.so > gpurun_out/r04e/lib_prev.log 2>&1 || exit 1
tail -3 gpurun_out/r04e/lib_prev.log
