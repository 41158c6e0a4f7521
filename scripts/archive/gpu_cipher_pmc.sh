# SQ counters of the BLAKE2b chunk-digest and AES-GCM kernels under scripts/gcm_probe.py (config 2
# chunks): instruction mix and busy cycles behind DESIGN.md §3b / §3c.  Each counter set in its
# own rocprofv3 pass, each under its own time limit.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/cipher_pmc
mkdir -p $out
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $set --kernel-include-regex "rc_b2_kernel|rc_gcm_kernel" --output-format csv -d $out/pmc_$i -o run -- \
    python3 scripts/gcm_probe.py > $out/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -n 5 $out/pmc_$i.log; exit 5; }
done
python3 scripts/pmc_by_kernel.py $out/pmc_* | tee $out/pmc_by_kernel.txt
