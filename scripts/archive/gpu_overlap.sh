# Round 3: pipelined steps (RC_PIPELINED: the chain on CU-masked reserved CUs beside the next
# step's tile kernel) -- CU-mask placement probe, GPU parity, one-allocation A/B per config,
# and the bench line in both modes.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/overlap
mkdir -p $out
export TMPDIR=/tmp
for r in 16 8; do
  timeout -k 10 60 ./scripts/ubench/cumask_probe $r > $out/cumask_$r.log 2>&1
  rc=$?; echo "cumask $r rc=$rc"; cat $out/cumask_$r.log
  [ $rc -eq 0 ] || exit $rc
done
if [ -z "${NOTEST:-}" ]; then
timeout -k 10 900 python -u -m pytest tests/test_gpu_overlap.py -x -v -p no:cacheprovider \
    --timeout 300 --timeout-method thread > $out/pytest_overlap.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $out/pytest_overlap.log
[ $rc -eq 0 ] || exit $rc
fi
for cfg in ${CFGS:-2 harness 3iii}; do
  case $cfg in
    2) S=${S2:-"seq p8 p16 p32"};;
    harness) S=${SH:-"seq p8 p16 p32"};;
    3iii) S=${S3:-"seq p16 p32 p64"};;
    4) S=${S4:-"seq p16"};;
    3ii) S=${S3ii:-"seq p16"};;
  esac
  timeout -k 10 300 python -u scripts/overlap_ab.py $cfg 4 $S > $out/ab_$cfg.log 2>&1
  rc=$?; echo "ab $cfg rc=$rc"; grep '^{' $out/ab_$cfg.log
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u bench.py > $out/bench_on.log 2>&1
rc=$?; echo "bench on rc=$rc"; tail -c 1500 $out/bench_on.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --pipeline off --cpu-streams 0 > $out/bench_off.log 2>&1
rc=$?; echo "bench off rc=$rc"; tail -c 600 $out/bench_off.log
exit $rc
