# Round 3: the tile kernel's work schedule on the 224 CUs of pipelined steps (tuned on 256 in
# round 3: 25 % static, 32-tile units) -- one allocation per config, settings alternating.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/sched224
mkdir -p $out
AB_STEPS=20 timeout -k 10 400 python -u scripts/overlap_ab.py 2 4 p32 p32@100:32 p32@400:32 p32@250:16 p32@250:64 p64 > $out/ab_2.log 2>&1
rc=$?; echo "ab 2 rc=$rc"; grep '^{' $out/ab_2.log
[ $rc -eq 0 ] || exit $rc
AB_STEPS=10 timeout -k 10 400 python -u scripts/overlap_ab.py 4 3 p32 p32@100:32 p32@250:64 > $out/ab_4.log 2>&1
rc=$?; echo "ab 4 rc=$rc"; grep '^{' $out/ab_4.log
exit $rc
