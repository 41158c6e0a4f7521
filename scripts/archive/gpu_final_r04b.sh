# Round 4 final validation, part 2: one bench line per BASELINE configuration (20 steps, the
# driver's count), a two-rank rehearsal on the one GPU (--share-gpus: every rank's parity), then
# the kernel trace + PMC passes of the default bench command (last: a profiler failure ends it).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final4
export TMPDIR=/tmp
# PART=configs: the bench lines only; PART=rest: the rehearsal and the profiler passes; unset: all
PART=${PART:-all}
CONFIG_ARGS=("--steps 20 --calibrate --e2e" "--steps 20 --config 3iii" "--steps 20 --config 3i" "--config 4 --steps 5 --warmup 1" "--steps 20 --key seeded --cpu-streams 0" "--steps 20 --config 3ii --cpu-streams 0" "--steps 20 --config 5 --cpu-streams 0" "--steps 20 --config harness" "--steps 20 --pipeline off --cpu-streams 0")
[ "$PART" = rest ] && CONFIG_ARGS=()
[ "$PART" = rest ] || : > gpurun_out/final4/configs.log
for args in "${CONFIG_ARGS[@]}"; do
  echo "== $args" | tee -a gpurun_out/final4/configs.log
  timeout -k 10 400 python bench.py $args >> gpurun_out/final4/configs.log 2>&1 || { echo "failed: $args"; tail -5 gpurun_out/final4/configs.log; exit 4; }
  tail -1 gpurun_out/final4/configs.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r['frac_read'], r['chain_kernel_ms'], d['parity_sha256'], d['pipeline'].get('pipelined_steps'), d['pipeline'].get('unpipelined_ms_per_step'), d.get('read_probe_gbs'), d.get('e2e_host_gibs'), (d.get('cpu_baseline') or {}).get('value'))"
done
[ "$PART" = configs ] && exit 0
echo "== --gpus 2 --share-gpus"
timeout -k 10 400 python bench.py --gpus 2 --share-gpus --steps 10 --cpu-streams 0 > gpurun_out/final4/ranks2.log 2>&1 || { echo "2-rank rehearsal failed"; tail -5 gpurun_out/final4/ranks2.log; exit 5; }
grep '^{' gpurun_out/final4/ranks2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['n_gpus'], d['ranks_seen'], d['distinct_devices'], d['parity_sha256'], [r['parity'] for r in d['per_rank']], d['pipeline'].get('pipelined_steps'))"
mkdir -p gpurun_out/prof
BENCH="bench.py --steps 5 --warmup 1 --cpu-streams 0 --no-verify"
# the trace pass at the driver's 20 steps (the average then carries one warm-up launch in 22)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/trace -o run -- python3 bench.py --steps 20 --warmup 2 --cpu-streams 0 --no-verify > gpurun_out/prof/trace.log 2>&1 || { echo trace failed; tail -20 gpurun_out/prof/trace.log; exit 6; }
grep '^{' gpurun_out/prof/trace.log | cut -c1-200
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "rc_tile|rc_read_probe" --output-format csv -d gpurun_out/prof/fetch -o run -- python3 $BENCH --calibrate > gpurun_out/prof/fetch.log 2>&1 || { echo "fetch pass failed rc=$?"; exit 7; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "rc_tile" --output-format csv -d gpurun_out/prof/write -o run -- python3 $BENCH > gpurun_out/prof/write.log 2>&1 || { echo "write pass failed rc=$?"; exit 7; }
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex "rc_tile" --output-format csv -d gpurun_out/prof/sq -o run -- python3 $BENCH > gpurun_out/prof/sq.log 2>&1 || { echo "sq pass failed rc=$?"; exit 7; }
echo "profile done"
