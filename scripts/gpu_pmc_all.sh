# rocprofv3 counters for EVERY BASELINE bench line: per workload a kernel
# trace (--kernel-trace --stats, the bench line with its build id), a FETCH_SIZE pass with the
# read probe over the same bytes (--calibrate: the calibration), a WRITE_SIZE pass; the harness
# and config 2 also an SQ pass (VALU issue, clock).  Each pass is its own run under its own time
# limit (MI355X_MICROARCH.md: never more counters than one pass holds); a failure ends the script.
# Summarise with:  for w in ...; do python scripts/summarize_profile.py r05 --workload $w gpurun_out/pmc/$w; done
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
ONLY=${ONLY:-}
COMMON="--steps 3 --warmup 1 --cpu-streams 0 --no-verify"
# (COMMON first: a workload's own --steps / --warmup win; the harness warms up as its bench line
# does, 50 steps -- its sub-millisecond launches run slower while the clock still ramps)
declare -A ARGS=([config2]="--config 2" [config2_seeded]="--config 2 --key seeded" [config3ii]="--config 3ii" [config3iii]="--config 3iii" [config4]="--config 4 --steps 2" [config5]="--config 5" [harness]="--config harness --warmup 50")
for w in config2 harness config3iii config3ii config5 config2_seeded config4; do
  [ -n "$ONLY" ] && [[ " $ONLY " != *" $w "* ]] && continue
  d=gpurun_out/pmc/$w
  mkdir -p $d
  A="$COMMON ${ARGS[$w]}"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $d/trace -o run -- python3 bench.py $A ${TRACE_STEPS:---steps 20} > $d/trace.log 2>&1 || { echo "$w trace failed"; tail -5 $d/trace.log; exit 5; }
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "rc_tile|rc_read_probe" --output-format csv -d $d/fetch -o run -- python3 bench.py $A --calibrate > $d/fetch.log 2>&1 || { echo "$w fetch failed"; tail -5 $d/fetch.log; exit 6; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "rc_tile" --output-format csv -d $d/write -o run -- python3 bench.py $A > $d/write.log 2>&1 || { echo "$w write failed"; tail -5 $d/write.log; exit 7; }
  if [ $w = harness ] || [ $w = config2 ]; then
    timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-include-regex "rc_tile" --output-format csv -d $d/sq -o run -- python3 bench.py $A > $d/sq.log 2>&1 || { echo "$w sq failed"; tail -5 $d/sq.log; exit 8; }
  fi
  echo "$w done: $(grep -h '^{' $d/trace.log | cut -c1-120)"
done
echo pmc done
