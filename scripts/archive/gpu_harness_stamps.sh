# Round 3: when the waves of the harness's tile kernel start and end (diag/lib_TSTAMPS.so), and
# the same for config 2, to see where the harness's short launch loses its rate.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/hstamps
mkdir -p $out
timeout -k 10 300 python -u scripts/tile_stamps.py harness > $out/harness.log 2>&1
rc=$?; echo "harness rc=$rc"; grep '^{' $out/harness.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/tile_stamps.py > $out/config2.log 2>&1
rc=$?; echo "config2 rc=$rc"; grep '^{' $out/config2.log
exit $rc
