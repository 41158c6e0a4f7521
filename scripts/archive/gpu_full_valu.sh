# gpu_full.sh, then the VALU issue/latency microbenchmark (scripts/ubench/valu_rates).
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_full.sh || exit $?
timeout -k 10 120 ./scripts/ubench/valu_rates > gpurun_out/full/valu_rates.log 2>&1
rc=$?; echo "valu rc=$rc"; cat gpurun_out/full/valu_rates.log
exit $rc
