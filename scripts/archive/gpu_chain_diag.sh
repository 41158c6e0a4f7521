# Chain-kernel diagnosis for one configuration: per-step stamps of one walker (diag build
# diag/lib_STAMPS.so), then PMC passes restricted to the chain kernels (--kernel-include-regex,
# so the fill and tile kernels are not counted).
#   ARGS="65536 1 2000 80000" CFG=3iii bash scripts/gpu_chain_diag.sh
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/chain_diag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python3 scripts/diag_stamps.py ${ARGS:-65536 1 2000 80000} > $out/stamps.log 2>&1 \
  || { echo "stamps failed"; tail -n 5 $out/stamps.log; exit 4; }
cat $out/stamps.log | tail -n 8
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-include-regex "${REGEX:-rc_spec_kernel}" --output-format csv -d $out/pmc_$tag -o run -- \
    python3 bench.py --config ${CFG:-3iii} --steps 2 --warmup 1 --cpu-streams 0 --no-verify > $out/pmc_$tag.log 2>&1 \
    || { echo "pmc $tag failed"; tail -n 5 $out/pmc_$tag.log; exit 5; }
done
python3 scripts/pmc_by_kernel.py $out/pmc_* | tee $out/pmc_by_kernel.txt
