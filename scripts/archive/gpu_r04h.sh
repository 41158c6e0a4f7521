# Round 4: RC_TILE_CLIP (a stream's last tile reads only its needed words) against the production
# build, both loaded in one process on one allocation per config (scripts/lib_ab.py; identical
# cut lists asserted).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04h
export TMPDIR=/tmp
for c in 3iii 2 harness; do
  timeout -k 10 300 python -u scripts/lib_ab.py $c 8 replicat_amd/libreplicat_chunker.so diag/lib_CLIP.so > gpurun_out/r04h/ab_$c.log 2>&1 || { echo "A/B $c failed"; tail -5 gpurun_out/r04h/ab_$c.log; exit 3; }
  tail -1 gpurun_out/r04h/ab_$c.log
done
