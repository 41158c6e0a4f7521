# Round 5, pass l: with workgroup grabs a late workgroup only takes later units, so fewer
# reserved CUs may no longer unbalance the shader engines -- pipelined steps on 8 / 16 / 32
# reserved CUs against sequential ones, config 2, the harness and 3 (ii), one allocation each.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05l
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/overlap_ab.py 2 3 p32 p16 p8 seq > $out/ab_c2.log 2>&1 || { echo "ab c2 failed"; tail -5 $out/ab_c2.log; exit 3; }
tail -1 $out/ab_c2.log
timeout -k 10 300 python -u scripts/overlap_ab.py harness 6 p32 p16 p8 seq > $out/ab_harness.log 2>&1 || { echo "ab harness failed"; tail -5 $out/ab_harness.log; exit 4; }
tail -1 $out/ab_harness.log
timeout -k 10 500 python -u scripts/overlap_ab.py 3ii 3 p32 p16 p8 seq > $out/ab_c3ii.log 2>&1 || { echo "ab 3ii failed"; tail -5 $out/ab_c3ii.log; exit 5; }
tail -1 $out/ab_c3ii.log
echo done
