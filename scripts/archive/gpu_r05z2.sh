# Round 5, pass z2: is the group records' cost the number of store bytes / instructions?  A
# timing-only build storing the first 16 of the 48 bytes (one store; the chain then works on
# partial ballots, so its cut lists are not compared) against the product, 3 (iii).
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r05z
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/lib_ab.py 3iii 4 diag/lib_NOTAIL_G16.so replicat_amd/libreplicat_chunker.so > $out/lib_ab_g16.log 2>&1 || { echo "lib ab g16 failed"; tail -5 $out/lib_ab_g16.log; exit 3; }
tail -1 $out/lib_ab_g16.log
echo done
