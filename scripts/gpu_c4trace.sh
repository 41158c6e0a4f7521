# Per-kernel durations for config 2 vs larger streams (kernel trace only, no counters).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c4t
export TMPDIR=/tmp
for spec in "c2:--config 2 --steps 5 --warmup 1" "c2_512x128:--config 2 --streams 512 --stream-mib 128 --steps 5 --warmup 1" "c4_8x8g:--config 4 --streams 8 --steps 5 --warmup 1"; do
  tag=${spec%%:*}; args=${spec#*:}
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4t/$tag -o run -- python3 bench.py --no-verify --cpu-streams 0 $args > gpurun_out/c4t/$tag.log 2>&1 || { echo "failed $tag"; tail -5 gpurun_out/c4t/$tag.log; exit 4; }
  echo "== $tag"; python3 scripts/kstats.py $(find gpurun_out/c4t/$tag -name '*kernel_stats.csv' | head -1)
done
