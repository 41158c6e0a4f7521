# Final validation (round 6: the maintained copy of archive/gpu_final_r05.sh): one bench line per BASELINE
# 20 steps (config 4: 5), each carrying rocprofv3 traffic from profiles/r06/pmc_summary.json of
# this same build, then a two-rank rehearsal on the one GPU (--share-gpus: every rank's parity).
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/final6
mkdir -p $out
export TMPDIR=/tmp
CONFIG_ARGS=("--steps 20 --calibrate --e2e" "--steps 20 --config 3iii" "--steps 20 --config 3i" "--config 4 --steps 5 --warmup 1" "--steps 20 --key seeded --cpu-streams 0" "--steps 20 --config 3ii --cpu-streams 0" "--steps 20 --config 5 --cpu-streams 0" "--steps 20 --config harness --calibrate" "--steps 20 --pipeline off --cpu-streams 0")
: > $out/configs.log
for args in "${CONFIG_ARGS[@]}"; do
  echo "== $args" | tee -a $out/configs.log
  timeout -k 10 400 python bench.py $args >> $out/configs.log 2>&1 || { echo "failed: $args"; tail -5 $out/configs.log; exit 4; }
  python3 scripts/final_table.py $out/configs.log | tail -1
done
echo "== --gpus 2 --share-gpus"
timeout -k 10 400 python bench.py --gpus 2 --share-gpus --steps 10 --cpu-streams 0 > $out/ranks2.log 2>&1 || { echo "2-rank rehearsal failed"; tail -5 $out/ranks2.log; exit 5; }
grep '^{' $out/ranks2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['n_gpus'], d['ranks_seen'], d['distinct_devices'], d['parity_sha256'], [r['parity'] for r in d['per_rank']], d['pipeline'].get('pipelined_steps'))"
echo done
