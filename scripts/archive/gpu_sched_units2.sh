# Round 3: dynamic unit size, second allocation -- 6 to 16 tiles per grab.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/sched_units2
mkdir -p $out
AB_STEPS=20 timeout -k 10 500 python -u scripts/overlap_ab.py 2 4 p32@250:32 p32@250:16 p32@250:12 p32@250:10 p32@250:8 p32@250:6 seq@250:12 seq@250:8 seq@250:6 > $out/ab_2.log 2>&1
rc=$?; echo "ab 2 rc=$rc"; grep '^{' $out/ab_2.log
[ $rc -eq 0 ] || exit $rc
AB_STEPS=20 timeout -k 10 500 python -u scripts/overlap_ab.py 3ii 3 p32@250:32 p32@250:12 p32@250:8 > $out/ab_3ii.log 2>&1
rc=$?; echo "ab 3ii rc=$rc"; grep '^{' $out/ab_3ii.log
exit $rc
