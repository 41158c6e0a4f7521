# Round 3: placement study step 2 and the digest-overlap queue hypothesis.
#   1. scripts/placement_probe2.py 6: one launch vs k launches, tile orders, per allocation
#   2. digest_overlap_probe.py with GPU_MAX_HW_QUEUES=8 (is 4 queues what caps 3-4 slots?)
#   3. one --pmc pass asking for TCC_EA0_RDREQ without _sum (per-channel rows or not?)
#   4. scripts/tile_stamps.py (diag/lib_TSTAMPS.so): when each tile-kernel wave ends
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/probe_c
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/placement_probe2.py 6 > $out/placement2.log 2>&1
rc=$?; echo "placement2 rc=$rc"; grep '^{' $out/placement2.log
[ $rc -eq 0 ] || exit $rc
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python -u scripts/digest_overlap_probe.py > $out/digest_overlap_q8.log 2>&1
rc=$?; echo "overlap q8 rc=$rc"; grep '^{' $out/digest_overlap_q8.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ -d $out/pmc_tcc -o run --output-format csv \
    -- python3 -u scripts/placement_probe2.py 1 > $out/pmc_tcc.log 2>&1
rc=$?; echo "pmc tcc rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/tile_stamps.py > $out/tile_stamps.log 2>&1
rc=$?; echo "stamps rc=$rc"; grep '^{' $out/tile_stamps.log | cut -c1-700
exit $rc
