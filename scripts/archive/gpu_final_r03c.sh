# Round 3, pipelined build (RC_PIPELINE_END): one bench line per BASELINE configuration
# (20 steps, the driver's count), a two-rank rehearsal on the one GPU (--share-gpus), then the
# kernel trace + PMC passes of the default bench command (last: a profiler failure ends it).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
CONFIG_ARGS_DEFAULT=("--steps 20 --calibrate --e2e" "--steps 20 --config 3iii" "--steps 20 --config 3i" "--config 4 --steps 5 --warmup 1" "--steps 20 --key seeded --cpu-streams 0" "--steps 20 --config 3ii --cpu-streams 0" "--steps 20 --config 5 --cpu-streams 0" "--steps 20 --config harness" "--steps 20 --pipeline off --cpu-streams 0")
: > gpurun_out/final/configs.log
for args in "${CONFIG_ARGS_DEFAULT[@]}"; do
  echo "== $args" | tee -a gpurun_out/final/configs.log
  timeout -k 10 400 python bench.py $args >> gpurun_out/final/configs.log 2>&1 || { echo "failed: $args"; tail -5 gpurun_out/final/configs.log; exit 4; }
  tail -1 gpurun_out/final/configs.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r['chain_kernel_ms'], d['parity_sha256'], d['pipeline'].get('pipelined_steps'), d['pipeline'].get('unpipelined_ms_per_step'), d.get('read_probe_gbs'), d.get('e2e_host_gibs'), (d.get('cpu_baseline') or {}).get('value'))"
done
echo "== --gpus 2 --share-gpus" | tee -a gpurun_out/final/configs.log
timeout -k 10 400 python bench.py --gpus 2 --share-gpus --steps 10 --cpu-streams 0 > gpurun_out/final/ranks2.log 2>&1 || { echo "2-rank rehearsal failed"; tail -5 gpurun_out/final/ranks2.log; exit 5; }
grep '^{' gpurun_out/final/ranks2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['n_gpus'], d['ranks_seen'], d['distinct_devices'], d['roofline'].get('frac'), d['parity_sha256'], d['pipeline'].get('pipelined_steps'))"
bash scripts/gpu_profile.sh
