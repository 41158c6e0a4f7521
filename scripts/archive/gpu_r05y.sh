# Round 5, pass y: timing events without the system-scope fence -- pipelined harness and
# config-2 steps with and without per-call timing on this library and the previous one
# (RC_LIB_PATH), then the GPU tests that read kernel timings and the two bench lines.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05y
mkdir -p $out
export TMPDIR=/tmp
for lib in new old; do
  if [ $lib = old ]; then export RC_LIB_PATH=diag/lib_pre_ev.so; else unset RC_LIB_PATH; fi
  for t in 1 0; do
    AB_STEPS=20 AB_TIMING=$t timeout -k 10 300 python -u scripts/overlap_ab.py harness 4 p32 > $out/ab_harness_${lib}_t$t.log 2>&1 || { echo "ab $lib t$t failed"; tail -5 $out/ab_harness_${lib}_t$t.log; exit 3; }
    echo "harness $lib timing=$t: $(tail -1 $out/ab_harness_${lib}_t$t.log | cut -c1-260)"
  done
done
unset RC_LIB_PATH
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_overlap.py tests/test_gpu_parity.py -k "pipelined or timing or harness or full_size" > $out/pytest.log 2>&1 || { echo "tests failed"; tail -30 $out/pytest.log; exit 4; }
tail -1 $out/pytest.log
timeout -k 10 300 python -u bench.py --config harness --steps 20 > $out/bench_harness.log 2>&1 || { echo "bench harness failed"; tail -5 $out/bench_harness.log; exit 5; }
tail -1 $out/bench_harness.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('harness', d['value'], d['ms_per_step'], r['kernel_ms'], d['warmup'], d['parity_sha256'], d['devices'])"
timeout -k 10 300 python -u bench.py --cpu-streams 0 > $out/bench_c2.log 2>&1 || { echo "bench c2 failed"; tail -5 $out/bench_c2.log; exit 6; }
tail -1 $out/bench_c2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('config2', d['value'], d['ms_per_step'], r['kernel_ms'], d['warmup'], d['parity_sha256'], d['devices'])"
echo done
