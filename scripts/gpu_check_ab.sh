# Chunker change check: parity tests, then an A/B against RC_LIB_PATH=$B on the same box.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TESTS="${TESTS:-tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_config4.py}" CONFIGS="" bash scripts/gpu_chunker_check.sh || exit $?
B=${B:-replicat_amd/diag_prev.so} CONFIGS="${CONFIGS:-2 3iii}" ROUNDS=${ROUNDS:-2} bash scripts/gpu_ab.sh
