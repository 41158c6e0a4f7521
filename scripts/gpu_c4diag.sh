# Config-4 slowdown attribution: tile kernel and read probe vs footprint and stream size.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c4
export TMPDIR=/tmp
run() {
  tag=$1; shift
  echo "== $tag: $*"
  timeout -k 10 240 python -u bench.py --no-verify --cpu-streams 0 --calibrate "$@" > gpurun_out/c4/$tag.log 2>&1 || { echo "failed $tag"; tail -5 gpurun_out/c4/$tag.log; exit 4; }
  tail -1 gpurun_out/c4/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms'], r['achieved'], r['chain_kernel_ms'], 'probe', d.get('read_probe_gbs'))"
}
run c2 --config 2 --steps 10 --warmup 2
run c2_2048x64 --config 2 --streams 2048 --steps 5 --warmup 1
run c2_512x128 --config 2 --streams 512 --stream-mib 128 --steps 10 --warmup 2
run c4 --config 4 --steps 3 --warmup 1
run c4_8x8g --config 4 --streams 8 --steps 5 --warmup 1
