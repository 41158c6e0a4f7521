# Chunker change check on one box: the chunker's GPU parity tests, then one bench line per
# configuration (parity flag in each line), then a kernel trace of each configuration.
#   TESTS="tests/test_gpu_parity.py" CONFIGS="3iii 2" TRACE="3iii" bash scripts/gpu_chunker_check.sh
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/check
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_large.py} -m gpu -x -q \
  -p no:cacheprovider --timeout 240 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
for cfg in ${CONFIGS:-3iii 2}; do
  timeout -k 10 300 python -u bench.py --config $cfg --steps ${STEPS:-10} --warmup 2 --cpu-streams 0 > $out/bench_$cfg.log 2>&1 \
    || { echo "bench $cfg failed"; tail -n 5 $out/bench_$cfg.log; exit 4; }
  tail -n 1 $out/bench_$cfg.log
done
for cfg in ${TRACE:-}; do
  t=$out/trace_$cfg
  mkdir -p $t
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $t -o run -- \
    python3 bench.py --config $cfg --steps 5 --warmup 1 --cpu-streams 0 --no-verify > $t/bench.log 2>&1 \
    || { echo "trace $cfg failed"; tail -n 20 $t/bench.log; exit 5; }
  python3 scripts/kstats.py "$(find $t -name '*kernel_stats.csv' | head -1)" | tee $t/kstats.txt
done
