# Round 5, pass x: does the bench's short warm-up leave the GPU below its clock? The harness and
# config 2 lines at several warm-up counts, one box.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05x
mkdir -p $out
export TMPDIR=/tmp
pr() { tail -1 $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms'], d['warmup'], d['devices'])"; }
for w in 2 50 200; do
  timeout -k 10 300 python -u bench.py --config harness --steps 20 --warmup $w --cpu-streams 0 > $out/harness_w$w.log 2>&1 || { echo "harness w$w failed"; tail -5 $out/harness_w$w.log; exit 3; }
  echo "harness w$w: $(pr $out/harness_w$w.log)"
done
for w in 2 10 30; do
  timeout -k 10 300 python -u bench.py --warmup $w --cpu-streams 0 > $out/c2_w$w.log 2>&1 || { echo "c2 w$w failed"; tail -5 $out/c2_w$w.log; exit 4; }
  echo "config2 w$w: $(pr $out/c2_w$w.log)"
done
echo done
