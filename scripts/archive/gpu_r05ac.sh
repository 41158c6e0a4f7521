# Round 5, pass ac: is rc_gcm_kernel's LDS array saturated?  SQ counters of the round-5 GCM kernel
# (and the BLAKE2b digests) under scripts/gcm_probe.py on config 2's chunks: LDS-array cycles
# (SQ_LDS_IDX_ACTIVE), bank conflicts, LDS and VALU instructions and their active cycles.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05ac
mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "rc_b2_kernel|rc_gcm_kernel" --output-format csv -d $out/pmc_1 -o run -- python3 scripts/gcm_probe.py > $out/pmc_1.log 2>&1 || { echo "pmc pass failed"; tail -n 8 $out/pmc_1.log; exit 5; }
python3 scripts/pmc_by_kernel.py $out/pmc_1 | tee $out/pmc_by_kernel.txt
tail -n 3 $out/pmc_1.log
