set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_v29.log 2>&1; rc=$?; tail -1 gpurun_out/bench_v29.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof29" -o bench -- python bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/prof29.log 2>&1; rc=$?; [ $rc -ne 0 ] && exit $rc
f=$(find gpurun_out/prof29 -name "*kernel_trace.csv" | head -1); python scripts/trace_gaps.py "$f" > gpurun_out/step_trace_v29.txt; tail -3 gpurun_out/step_trace_v29.txt
