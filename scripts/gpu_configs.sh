# One bench line per configuration (BASELINE.json configs 2, 3i, 3ii, 3iii, 4, 5, the reference harness) + calibration/e2e.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/configs.log
for args in ${CONFIG_ARGS:-"--calibrate --e2e" "--config 3iii" "--config 3i" "--config 4 --steps 3 --warmup 1" "--key seeded --cpu-streams 0" "--config 3ii --cpu-streams 0" "--config 5 --cpu-streams 0" "--config harness"}; do
  echo "== $args" | tee -a gpurun_out/configs.log
  timeout -k 10 400 python bench.py $args >> gpurun_out/configs.log 2>&1 || { echo "failed: $args"; tail -5 gpurun_out/configs.log; exit 4; }
  tail -1 gpurun_out/configs.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['chain_kernel_ms'], d['parity_sha256'], d.get('read_probe_gbs'), d.get('e2e_host_gibs'), (d.get('cpu_baseline') or {}).get('value'))"
done
