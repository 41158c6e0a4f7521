# Round 3: the producer with three batches in flight, and the placement study.
#   1. tests/test_gpu_pipeline.py (the producer, now `slots` batches in flight)
#   2. scripts/digest_overlap_probe.py: device-side per-batch work at 1-4 streams
#   3. scripts/placement_probe.py: fresh allocations (torch / contiguous), whole + per-4-GiB reads
#   4. the same under rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum
#   5. scripts/producer_probe.py 8192 128: 8 GiB of 64 MiB files end to end
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/probe_b
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py -x -v -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $out/pytest_pipeline.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest_pipeline.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/digest_overlap_probe.py > $out/digest_overlap.log 2>&1
rc=$?; echo "overlap rc=$rc"; cat $out/digest_overlap.log | grep '^{'
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/placement_probe.py 4 torch,contiguous > $out/placement.log 2>&1
rc=$?; echo "placement rc=$rc"; grep '^{' $out/placement.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum \
    -d $out/pmc_tlb -o run --output-format csv -- python3 -u scripts/placement_probe.py 3 torch,contiguous \
    > $out/placement_pmc.log 2>&1
rc=$?; echo "placement pmc rc=$rc"; grep '^{' $out/placement_pmc.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/producer_probe.py 8192 128 > $out/producer_8g.log 2>&1
rc=$?; echo "producer rc=$rc"; grep '^{' $out/producer_8g.log | cut -c1-400
exit $rc
