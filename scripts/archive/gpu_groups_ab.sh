# Round 3: config 3 (iii)'s tile-kernel cost split -- group records vs stream layout.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/groups_ab
mkdir -p $out
timeout -k 10 500 python -u scripts/groups_ab.py 4 > $out/ab.log 2>&1
rc=$?; echo "ab rc=$rc"; grep '^{' $out/ab.log
exit $rc
