# round 6: where the reference harness's short tile launch loses time -- every wave's start and
# end (TSTAMPS build) under the default schedule and smaller units / groups, then the product
# library on the same settings; config 2's default for comparison
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06l; mkdir -p $out
export TMPDIR=/tmp
RC_LIB_PATH=diag/lib_TSTAMPS.so timeout -k 10 300 python -u scripts/harness_sched_probe.py harness 4 0:3:0:64 0:2:0:16 0:3:0:16 0:2:0:64 > $out/harness_stamps.log 2>&1 || { tail -5 $out/harness_stamps.log; exit 3; }
tail -1 $out/harness_stamps.log
timeout -k 10 300 python -u scripts/harness_sched_probe.py harness 6 0:3:0:64 0:2:0:16 0:3:0:16 > $out/harness_sched.log 2>&1 || { tail -5 $out/harness_sched.log; exit 4; }
tail -1 $out/harness_sched.log
RC_LIB_PATH=diag/lib_TSTAMPS.so timeout -k 10 300 python -u scripts/harness_sched_probe.py 2 2 0:3:0:64 > $out/c2_stamps.log 2>&1 || { tail -5 $out/c2_stamps.log; exit 5; }
tail -1 $out/c2_stamps.log
