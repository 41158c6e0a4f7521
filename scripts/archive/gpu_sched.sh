# Round 3: tile-kernel schedule A/B on one allocation per config (scripts/tile_sched_ab.py), after
# the chunker parity tests on the same build.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/sched
mkdir -p $out
export TMPDIR=/tmp
if [ -z "${NOTEST:-}" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lane_chain.py \
    tests/test_gpu_harness.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread \
    > $out/pytest_chunker.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest_chunker.log
[ $rc -eq 0 ] || exit $rc
fi
for cfg in ${CFGS:-2 harness 3iii}; do
  case $cfg in
    2) S=${S2:-"1000:32 750:32 500:32 500:16 750:64 1000:32:g 750:32:g"};;
    harness) S=${SH:-"1000:32 750:32 500:32 250:32 1000:32:g 750:32:g"};;
    3iii) S=${S3:-"1000:32 750:32 500:32 500:16"};;
    4) S=${S4:-"1000:32 500:32"};;
  esac
  timeout -k 10 300 python -u scripts/tile_sched_ab.py $cfg 6 $S > $out/ab_$cfg.log 2>&1
  rc=$?; echo "ab $cfg rc=$rc"; grep '^{' $out/ab_$cfg.log
  [ $rc -eq 0 ] || exit $rc
done
exit 0
