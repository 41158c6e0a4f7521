# round 6 (second pass): the ring depth against waves per CU, beside the cache policy -- the tile kernel's streaming pattern with every policy
# bit combination of its buffer loads (scripts/ubench/ring_policy.hip -> diag/ring_policy)
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06s; mkdir -p $out
timeout -k 10 300 diag/ring_policy > $out/ring_policy.log 2>&1 || { cat $out/ring_policy.log; exit 3; }
cat $out/ring_policy.log
