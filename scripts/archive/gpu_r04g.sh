# Round 4: two alternating tile streams (RC_TILE_STREAMS=2) against one, pipelined, on one
# allocation per config (scripts/overlap_ab.py; wall ms per step is the comparison -- with two
# streams a tile kernel's HIP-event time includes the wait for the previous one's CUs).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04g
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/overlap_ab.py harness 6 p32 p32x2 p32x2@100:12:0 p32x2@250:8:0 > gpurun_out/r04g/ab_harness.log 2>&1 || { echo "harness A/B failed"; tail -5 gpurun_out/r04g/ab_harness.log; exit 3; }
tail -1 gpurun_out/r04g/ab_harness.log
timeout -k 10 400 python -u scripts/overlap_ab.py 2 6 p32 p32x2 > gpurun_out/r04g/ab_2.log 2>&1 || { echo "config 2 A/B failed"; tail -5 gpurun_out/r04g/ab_2.log; exit 4; }
tail -1 gpurun_out/r04g/ab_2.log
timeout -k 10 400 python -u scripts/overlap_ab.py 3ii 4 p32 p32x2 > gpurun_out/r04g/ab_3ii.log 2>&1 || { echo "3ii A/B failed"; tail -5 gpurun_out/r04g/ab_3ii.log; exit 5; }
tail -1 gpurun_out/r04g/ab_3ii.log
