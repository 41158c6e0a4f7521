# Round 3: the harness's launch (76 tiles per wave, static today) on the dynamic schedule with
# small units (RC_TILE_DYN_MIN=0 lets any launch hand out units), one allocation.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/harness_dyn
mkdir -p $out
RC_TILE_DYN_MIN=0 timeout -k 10 400 python -u scripts/tile_sched_ab.py harness 6 1000:12 100:12 0:12 0:8 0:4 250:8 > $out/ab_harness.log 2>&1
rc=$?; echo "ab rc=$rc"; grep '^{' $out/ab_harness.log
exit $rc
