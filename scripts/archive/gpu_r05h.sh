# Round 5, pass h: config 2's 0.7 % against round 4 -- the libraries of round 4, of 5aefdcb, of
# HEAD without the slice fence (diag NOFENCE) and HEAD on one allocation; the harness pipelined
# and in sequence with workgroup grabs (and two tile streams); config 2 under workgroup grabs.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05h
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/lib_ab.py 2 4 diag/lib_r04.so diag/lib_5aefdcb.so diag/lib_NOFENCE.so replicat_amd/libreplicat_chunker.so > $out/lib_ab_2.log 2>&1 || { echo "lib ab 2 failed"; tail -5 $out/lib_ab_2.log; exit 3; }
tail -1 $out/lib_ab_2.log
RC_TILE_STATIC=0 RC_TILE_CHUNK=3 RC_TILE_DYN_MIN=0 RC_TILE_GROUP=64 timeout -k 10 300 python -u scripts/lib_ab.py harness 6 diag/lib_NOFENCE.so replicat_amd/libreplicat_chunker.so > $out/lib_ab_harness_g64.log 2>&1 || { echo "lib ab harness failed"; tail -5 $out/lib_ab_harness_g64.log; exit 4; }
tail -1 $out/lib_ab_harness_g64.log
timeout -k 10 400 python -u scripts/overlap_ab.py harness 6 seq seq@0:3:0:64 p32 p32@0:3:0:64 p32@100:3:0:64 p32x2@0:3:0:64 p32x2 > $out/ab_harness.log 2>&1 || { echo "ab harness failed"; tail -5 $out/ab_harness.log; exit 5; }
tail -1 $out/ab_harness.log
timeout -k 10 500 python -u scripts/harness_sched_probe.py 2 3 100:12:128:0 100:12:0:32 100:6:0:32 100:4:0:64 100:3:0:64 0:3:0:64 > $out/c2_sched.log 2>&1 || { echo "c2 sched failed"; tail -5 $out/c2_sched.log; exit 6; }
tail -1 $out/c2_sched.log
echo done
