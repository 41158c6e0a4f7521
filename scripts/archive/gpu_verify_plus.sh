# gpu_verify.sh (the whole GPU suite, smoke, the default bench line), then on the same box:
#   lib_ab.py: this build vs the round-2 build (diag/lib_prev.so) on one allocation, configs 2, 3iii;
#   harness_chain_ab.py: the harness stream's segment length / extension.
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_verify.sh || exit $?
out=gpurun_out/verify
timeout -k 10 300 python -u scripts/lib_ab.py 2 6 replicat_amd/libreplicat_chunker.so diag/lib_prev.so > $out/lib_ab_2.log 2>&1
rc=$?; echo "lib_ab 2 rc=$rc"; grep '^{' $out/lib_ab_2.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/lib_ab.py 3iii 6 replicat_amd/libreplicat_chunker.so diag/lib_prev.so > $out/lib_ab_3iii.log 2>&1
rc=$?; echo "lib_ab 3iii rc=$rc"; grep '^{' $out/lib_ab_3iii.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/harness_chain_ab.py 5 > $out/harness_chain.log 2>&1
rc=$?; echo "harness chain rc=$rc"; grep '^{' $out/harness_chain.log
exit $rc
