# The device snapshot producer: its GPU parity tests, then the probe (config 1 = one 256 MiB
# file; 64 files / 4 GiB) for this tree and, if present, the round-1 producer on the same box.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/producer
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_snapshot.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
for args in ${PROBE_ARGS:-"256 1" "4096 64"}; do
  timeout -k 10 300 python -u scripts/producer_probe.py $args > "$out/probe_${args// /_}.log" 2>&1 || { echo "probe $args failed"; tail -20 "$out/probe_${args// /_}.log"; exit 3; }
  cat "$out/probe_${args// /_}.log" | grep -v amdgpu.ids
  if [ -f replicat_amd/_pipeline_r01.py ]; then
    RC_PRODUCER_MODULE=replicat_amd._pipeline_r01 timeout -k 10 300 python -u scripts/producer_probe.py $args > "$out/probe_r01_${args// /_}.log" 2>&1 || { echo "r01 probe $args failed"; exit 4; }
    grep -v amdgpu.ids "$out/probe_r01_${args// /_}.log" | sed 's/^/r01 /'
  fi
done
