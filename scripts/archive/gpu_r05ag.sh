# Round 5, pass ag: what in 3 (iii)'s pipelined chain slows the tile kernel beside it?  A
# timing-only build whose quad chain reads no stream words (diag/lib_NOWORDS.so: records only,
# wrong cuts) against the product, both pipelined (RC_PIPE_ALL=1, RC_PIPELINED calls), then the
# product in sequence for reference.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05ag
mkdir -p $out
export TMPDIR=/tmp
RC_PIPE_ALL=1 LIB_AB_FLAGS=2 timeout -k 10 400 python -u scripts/lib_ab.py 3iii 4 diag/lib_NOWORDS.so replicat_amd/libreplicat_chunker.so > $out/ab_piped.log 2>&1 || { echo "ab piped failed"; tail -5 $out/ab_piped.log; exit 3; }
tail -1 $out/ab_piped.log
timeout -k 10 400 python -u scripts/lib_ab.py 3iii 4 diag/lib_NOWORDS.so replicat_amd/libreplicat_chunker.so > $out/ab_seq.log 2>&1 || { echo "ab seq failed"; tail -5 $out/ab_seq.log; exit 4; }
tail -1 $out/ab_seq.log
echo done
