# Round 5, pass j: under the workgroup-grab default -- config 3 (iii) pipelined on 16 / 32 / 64
# reserved CUs against in sequence (RC_PIPE_ALL=1), 3 (iii) against config 2 on one allocation,
# the harness with one and two tile streams, and the harness / 3 (iii) bench lines.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05j
mkdir -p $out
export TMPDIR=/tmp
RC_PIPE_ALL=1 timeout -k 10 500 python -u scripts/overlap_ab.py 3iii 3 seq p16 p32 p64 > $out/ab_3iii.log 2>&1 || { echo "ab 3iii failed"; tail -5 $out/ab_3iii.log; exit 3; }
tail -1 $out/ab_3iii.log
timeout -k 10 500 python -u scripts/c2_vs_3iii.py 3 10 > $out/c2_vs_3iii.log 2>&1 || { echo "c2 vs 3iii failed"; tail -5 $out/c2_vs_3iii.log; exit 4; }
tail -1 $out/c2_vs_3iii.log
timeout -k 10 300 python -u scripts/overlap_ab.py harness 6 p32 p32x2 p16 p16x2 seq > $out/ab_harness.log 2>&1 || { echo "ab harness failed"; tail -5 $out/ab_harness.log; exit 5; }
tail -1 $out/ab_harness.log
timeout -k 10 300 python -u bench.py --config harness --steps 20 --warmup 3 > $out/bench_harness.log 2>&1 || { echo "bench harness failed"; tail -5 $out/bench_harness.log; exit 6; }
tail -1 $out/bench_harness.log | cut -c1-300
timeout -k 10 400 python -u bench.py --config 3iii > $out/bench_3iii.log 2>&1 || { echo "bench 3iii failed"; tail -5 $out/bench_3iii.log; exit 7; }
tail -1 $out/bench_3iii.log | cut -c1-300
echo done
PROBE_VARIANTS=plain,stream_release,stream_release_timeline,stream_release_3_slots_timeline timeout -k 10 400 python -u scripts/producer_probe.py 8192 128 > $out/producer.log 2>&1 || { echo "producer failed"; tail -5 $out/producer.log; exit 8; }
grep -h '"variant"' $out/producer.log | cut -c1-400
echo done2
