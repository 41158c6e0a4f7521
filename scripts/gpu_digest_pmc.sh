set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dpmc
export TMPDIR=/tmp
for N in 16384 32768; do
  export N_LIST=$N
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_IFETCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/dpmc/sq_$N -o run -- python3 scripts/digest_latency.py 1048576 > gpurun_out/dpmc/sq_$N.log 2>&1 || { echo "sq $N failed"; tail -5 gpurun_out/dpmc/sq_$N.log; exit 3; }
  timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/dpmc/ic_$N -o run -- python3 scripts/digest_latency.py 1048576 > gpurun_out/dpmc/ic_$N.log 2>&1 || { echo "ic $N failed"; tail -5 gpurun_out/dpmc/ic_$N.log; exit 4; }
done
find gpurun_out/dpmc -name "*counter_collection.csv" | head
