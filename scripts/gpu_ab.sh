# A/B of two chunker builds on one box: bench lines alternating between the in-tree library
# and RC_LIB_PATH=$B (default replicat_amd/diag_head.so), then optional PMC passes.
#   CONFIGS="2 3iii" ROUNDS=3 PMC_CONFIG=3iii bash scripts/gpu_ab.sh
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/ab
mkdir -p $out
export TMPDIR=/tmp
B=${B:-replicat_amd/diag_head.so}
for r in $(seq ${ROUNDS:-3}); do
  for cfg in ${CONFIGS:-2 3iii}; do
    order="new old"; [ $((r % 2)) -eq 0 ] && order="old new"   # alternate which runs first
    for v in $order; do
      if [ $v = old ]; then export RC_LIB_PATH=$B; else unset RC_LIB_PATH; fi
      timeout -k 10 300 python -u bench.py --config $cfg --steps 10 --warmup 2 --cpu-streams 0 --no-verify > $out/${v}_${cfg}_$r.log 2>&1 \
        || { echo "bench $v $cfg failed"; tail -n 5 $out/${v}_${cfg}_$r.log; exit 4; }
      tail -n 1 $out/${v}_${cfg}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', '$cfg', d['value'], d['ms_per_step'], r['kernel_ms'], r['edge_kernel_ms'], r['chain_kernel_ms'])"
    done
  done
done
unset RC_LIB_PATH
if [ -n "${PMC_CONFIG:-}" ]; then
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
    tag=$(echo $set | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $out/pmc_$tag -o run -- \
      python3 bench.py --config $PMC_CONFIG --steps 2 --warmup 1 --cpu-streams 0 --no-verify > $out/pmc_$tag.log 2>&1 \
      || { echo "pmc $tag failed"; tail -n 5 $out/pmc_$tag.log; exit 5; }
  done
  python3 scripts/pmc_by_kernel.py $out/pmc_* | tee $out/pmc_by_kernel.txt
fi
