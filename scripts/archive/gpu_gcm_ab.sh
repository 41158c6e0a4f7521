# AES-GCM: the cipher's GPU parity tests, then the config-2 encrypted-leg probe for this build
# and for RC_LIB_PATH=diag/lib_head.so (the previous build), alternated on one box; then a
# two-rank rehearsal of bench.py's multi-process path (both ranks on the box's one GPU).
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/gcm
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_gcm.py tests/test_gpu_pipeline.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in new head; do
    if [ $v = head ]; then export RC_LIB_PATH=diag/lib_head.so; else unset RC_LIB_PATH; fi
    timeout -k 10 300 python -u scripts/gcm_probe.py > $out/probe_${v}_$i.log 2>&1 || { echo "probe $v failed"; tail -20 $out/probe_${v}_$i.log; exit 3; }
    echo "$v $i: $(grep -v amdgpu.ids $out/probe_${v}_$i.log | tail -3 | tr '\n' ' ')"
  done
done
unset RC_LIB_PATH
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 > $out/bench_2ranks.log 2>&1
rc=$?; echo "2-rank bench rc=$rc"; grep -v amdgpu.ids $out/bench_2ranks.log | tail -3
exit $rc
