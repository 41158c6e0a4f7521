# Round 5, pass t: the fresh-chunker first-call test, the harness line with its read-probe
# ceiling (--calibrate), and 3 (iii) against config 2 on one allocation, on the final build.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05t
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_schedule.py -k fresh > $out/pytest.log 2>&1 || { echo "test failed"; tail -30 $out/pytest.log; exit 3; }
tail -1 $out/pytest.log
timeout -k 10 300 python -u bench.py --config harness --steps 20 --calibrate > $out/bench_harness.log 2>&1 || { echo "bench harness failed"; tail -5 $out/bench_harness.log; exit 4; }
tail -1 $out/bench_harness.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms'], r.get('frac'), r.get('traffic'), d.get('read_probe_gbs'), d['pipeline'].get('unpipelined_ms_per_step'), d['parity_sha256'], d['devices'])"
timeout -k 10 500 python -u scripts/c2_vs_3iii.py 3 10 > $out/c2_vs_3iii.log 2>&1 || { echo "c2 vs 3iii failed"; tail -5 $out/c2_vs_3iii.log; exit 5; }
tail -1 $out/c2_vs_3iii.log
echo done
timeout -k 10 200 python -u scripts/tile_stamps.py harness > $out/stamps_seq.log 2>&1 || { echo "stamps seq failed"; tail -5 $out/stamps_seq.log; exit 6; }
grep '"rep": 3' $out/stamps_seq.log
STAMPS_PIPE=32 timeout -k 10 200 python -u scripts/tile_stamps.py harness > $out/stamps_p32.log 2>&1 || { echo "stamps p32 failed"; tail -5 $out/stamps_p32.log; exit 7; }
grep '"rep": 3' $out/stamps_p32.log
echo done2
