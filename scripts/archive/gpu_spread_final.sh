# Round 3 final build: the allocation spread -- 3 processes x 3 fresh 64 GiB allocations, each
# timed with the config-2 tile kernel and the streaming read probe (scripts/placement_probe.py).
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/spread
mkdir -p $out
for p in 0 1 2; do
  timeout -k 10 300 python -u scripts/placement_probe.py 3 torch > $out/proc$p.log 2>&1 || { echo "placement $p failed"; tail -5 $out/proc$p.log; exit 4; }
  grep '^{' $out/proc$p.log | python3 -c "import json,sys; [print(d['rep'], d['tile_ms'], d['probe_gbs']) for d in map(json.loads, sys.stdin)]"
done
