# Round 3: segment floor / extension defaults with boundary repair (chain phase on one
# allocation per config, scripts/chain_ab.py; sequential calls).
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/repair2
mkdir -p $out
run() {  # log config settings...
  local log=$1; shift
  timeout -k 10 300 python -u scripts/chain_ab.py "$@" > $out/$log.log 2>&1
  local rc=$?; echo "ab $log rc=$rc"; grep '^{' $out/$log.log
  return $rc
}
run harness harness 4 f3:4 f3:4:norepair f3:2 f2:2 f2:3 f2:4 f3:3 && \
run 3ii 3ii 4 0:4 0:4:norepair 0:3 0:2 0:1 && \
run c4 4 3 0:4 0:2 && \
run c2 2 3 0:4 0:2
