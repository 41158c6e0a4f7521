# round 6: where the harness's pipelined step spends the ~0.02 ms beyond its tile kernel -- a
# rocprofv3 kernel trace of the harness line (gaps between consecutive tile kernels per queue)
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r06o; mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- python3 bench.py --config harness --steps 20 --cpu-streams 0 > $out/trace.log 2>&1 || { tail -5 $out/trace.log; exit 3; }
tail -1 $out/trace.log | cut -c1-300
f=$(find $out/trace -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_gaps.py $f rc_tile_kernel > $out/gaps.txt 2>&1 || { tail -5 $out/gaps.txt; exit 4; }
tail -40 $out/gaps.txt
