# Round 5, pass ab: SQ counters (VALU issue, LDS, clock) of config 3 (iii)'s tile kernel
# (rc_tile_kernel<4>), in sequence (its bench line) and pipelined (RC_PIPE_ALL=1: 224 CUs), to
# set beside config 2's rc_tile_kernel<1> in pmc_summary.json.  Same build as the summary.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
A="--steps 3 --warmup 1 --cpu-streams 0 --no-verify --config 3iii"
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
d=gpurun_out/pmc/config3iii
mkdir -p $d
timeout -s KILL 240 rocprofv3 --pmc $SQ --kernel-include-regex "rc_tile" --output-format csv -d $d/sq -o run -- python3 bench.py $A > $d/sq.log 2>&1 || { echo "sq failed"; tail -5 $d/sq.log; exit 3; }
echo "seq: $(grep -h '^{' $d/sq.log | cut -c1-160)"
p=gpurun_out/pmc/config3iii_piped
mkdir -p $p
RC_PIPE_ALL=1 timeout -s KILL 240 rocprofv3 --pmc $SQ --kernel-include-regex "rc_tile" --output-format csv -d $p/sq -o run -- python3 bench.py $A > $p/sq.log 2>&1 || { echo "sq piped failed"; tail -5 $p/sq.log; exit 4; }
echo "piped: $(grep -h '^{' $p/sq.log | cut -c1-160)"
echo done
