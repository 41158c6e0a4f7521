# Round 3: the default bench line (20 steps) and the kernel trace + PMC passes at the final
# build (scripts/gpu_profile.sh, last).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/final/bench.log 2>&1 || { echo bench failed; tail -5 gpurun_out/final/bench.log; exit 3; }
tail -1 gpurun_out/final/bench.log | cut -c1-300
bash scripts/gpu_profile.sh
