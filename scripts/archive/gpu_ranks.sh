# Round 3: bench.py --gpus N as its own launcher, on the one-GPU lease, plus the parity tests
# that used to live only in bench lines (harness, config 3 (i) full size, seeded key).
#   1. pytest tests/test_gpu_harness.py
#   2. bench.py --gpus 2 (no --share-gpus): must refuse (two ranks, one device) -- exit != 0
#   3. bench.py --gpus 2 --share-gpus: the rehearsal line, roofline null, two ranks seen
#   4. bench.py --key seeded: the encrypted-repository line with its parity flag
#   5. bench.py (the driver's command)
#   6. scripts/dropin_probe.py; 7. rocprofv3 --list-avail
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/ranks
mkdir -p $out
export TMPDIR=/tmp
fatal() { case $1 in 124|134|137|139) echo "fatal rc=$1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_harness.py -x -v -p no:cacheprovider \
    --timeout 300 --timeout-method thread > $out/pytest_harness.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $out/pytest_harness.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --gpus 2 --steps 3 --warmup 1 --cpu-streams 0 \
    > $out/refuse.log 2>&1
rc=$?; echo "refuse rc=$rc (expected non-zero)"; tail -3 $out/refuse.log
fatal $rc refuse
[ $rc -ne 0 ] || exit 9
timeout -k 10 400 python -u bench.py --gpus 2 --share-gpus --steps 5 --warmup 2 --cpu-streams 32 \
    > $out/share2.log 2>&1
rc=$?; echo "share rc=$rc"; tail -1 $out/share2.log | cut -c1-600
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --key seeded --cpu-streams 0 > $out/seeded.log 2>&1
rc=$?; echo "seeded rc=$rc"; tail -1 $out/seeded.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $out/bench.log | cut -c1-400
[ $rc -eq 0 ] || exit $rc
#   6. the drop-in path: replicat's adapter loop over the HIP _gclmulchunker vs the reference .so
timeout -k 10 400 python -u scripts/dropin_probe.py --repeat 2 > $out/dropin.log 2>&1
rc=$?; echo "dropin rc=$rc"; cut -c1-600 $out/dropin.log | tail -3
[ $rc -eq 0 ] || exit $rc
#   7. the counters this box offers (per-channel TCC instances for the placement study)
timeout -k 10 120 rocprofv3 --list-avail > $out/counters.txt 2>&1
echo "list rc=$?"
exit 0
