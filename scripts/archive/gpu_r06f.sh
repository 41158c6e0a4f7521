# round 6: 3 (iii) pipelined vs in sequence with the SDWA tile kernel (no runner-up bounds):
# overlap_ab on one allocation, RC_PIPE_ALL=1 so that the small-window request overlaps
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06f; mkdir -p $out
export TMPDIR=/tmp
RC_LIB_PATH=diag/lib_sdwa.so RC_PIPE_ALL=1 timeout -k 10 300 python -u scripts/overlap_ab.py 3iii 4 seq p32 p64 > $out/overlap_3iii_sdwa.log 2>&1; tail -1 $out/overlap_3iii_sdwa.log
RC_LIB_PATH=diag/lib_base6.so RC_PIPE_ALL=1 timeout -k 10 300 python -u scripts/overlap_ab.py 3iii 4 seq p32 > $out/overlap_3iii_base6.log 2>&1; tail -1 $out/overlap_3iii_base6.log
