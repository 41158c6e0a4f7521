# round 6: config 3 (iii) pipelined -- does the chain's scatter slow the tile kernel beside it?
# The product against a timing-only build whose quad chain reads each task's 64 bytes
# consecutively (diag/lib_NOWORDS_CONTIG.so, -DRC_DIAG_CHAIN_CONTIG), on one allocation,
# pipelined (RC_PIPE_ALL=1, flags 2) and in sequence
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06m; mkdir -p $out
export TMPDIR=/tmp
RC_PIPE_ALL=1 LIB_AB_FLAGS=2 timeout -k 10 300 python -u scripts/lib_ab.py 3iii 6 replicat_amd/libreplicat_chunker.so diag/lib_NOWORDS_CONTIG.so > $out/ab_piped.log 2>&1 || { tail -5 $out/ab_piped.log; exit 3; }
tail -1 $out/ab_piped.log
timeout -k 10 300 python -u scripts/lib_ab.py 3iii 6 replicat_amd/libreplicat_chunker.so diag/lib_NOWORDS_CONTIG.so > $out/ab_seq.log 2>&1 || { tail -5 $out/ab_seq.log; exit 4; }
tail -1 $out/ab_seq.log
