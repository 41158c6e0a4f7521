# Bench under several environment settings (one process each, each under its own limit).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/sweep.log
for spec in "$@"; do
  echo "== $spec" | tee -a gpurun_out/sweep.log
  env $spec timeout -k 10 300 python bench.py --steps 10 --warmup 2 --cpu-streams 0 ${BENCH_ARGS:-} >> gpurun_out/sweep.log 2>&1 || { echo "failed: $spec"; exit 4; }
  tail -1 gpurun_out/sweep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline'] or {}; print(d['value'], d['ms_per_step'], r.get('kernel_ms'), r.get('edge_kernel_ms'), r.get('chain_kernel_ms'), d['parity_sha256'], d.get('read_probe_gbs'))"
done
