# round 6: what the tile kernel's auxiliary loads cost (the word before each tile, the retire's
# candidate words): the product against a timing-only build that loads them from one hot address
# (diag/lib_NOEXACT_AUXHOT.so, -DRC_DIAG_AUX_HOT), one allocation, config 2 and the harness (first pipelined, then -- this version -- in sequence, so that the timing build's slow chains run after its tile kernels)
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06p; mkdir -p $out
export TMPDIR=/tmp
LIB_AB_FLAGS=0 timeout -k 10 400 python -u scripts/lib_ab.py 2 8 replicat_amd/libreplicat_chunker.so diag/lib_NOEXACT_AUXHOT.so > $out/ab_c2_seq.log 2>&1 || { tail -5 $out/ab_c2_seq.log; exit 3; }
tail -1 $out/ab_c2_seq.log
LIB_AB_FLAGS=0 timeout -k 10 300 python -u scripts/lib_ab.py harness 12 replicat_amd/libreplicat_chunker.so diag/lib_NOEXACT_AUXHOT.so > $out/ab_h_seq.log 2>&1 || { tail -5 $out/ab_h_seq.log; exit 4; }
tail -1 $out/ab_h_seq.log
