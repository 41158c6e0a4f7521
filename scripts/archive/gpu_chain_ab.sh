# Chain-kernel variants (record-cache rows RC_REC_UNROLL, edge-scan batch RC_EDGE_ITERS) against
# the default build, same allocation, one process per configuration (scripts/lib_ab.py).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/chain_ab
LIBS="replicat_amd/libreplicat_chunker.so ${VARIANTS:-diag/lib_REC5.so diag/lib_E4.so diag/lib_R5E4.so diag/lib_E8.so}"
for cfg in ${CFGS:-2 harness 3ii 4}; do
  timeout -k 10 300 python -u scripts/lib_ab.py $cfg ${ROUNDS:-6} $LIBS > gpurun_out/chain_ab/ab_$cfg.log 2>&1 || { echo "ab $cfg failed"; tail -5 gpurun_out/chain_ab/ab_$cfg.log; exit 1; }
  grep '^{' gpurun_out/chain_ab/ab_$cfg.log
done
