#!/bin/bash
# Round 5: where the host's time goes in the bench step (host_split: the post-read-back host segment; cProfile of 50
# steps), with a kernel trace of the driver's command for the idle gaps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r5j}"; mkdir -p "$O"
timeout -k 10 200 python scripts/host_split.py --steps 40 > "$O/host_split.txt" 2>&1 || { tail -20 "$O/host_split.txt"; exit 1; }
grep -v amdgpu "$O/host_split.txt"
timeout -k 10 200 python scripts/host_profile.py > "$O/host_profile.txt" 2>&1 || { tail -20 "$O/host_profile.txt"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof" -o run -- python3 bench.py --gpus 1 --steps 20 \
    --warmup 5 --cpu-baseline off > "$O/bench_prof.log" 2>&1 || { tail -20 "$O/bench_prof.log"; exit 1; }
f=$(find "$O/prof" -name '*kernel_trace.csv' | head -1); cp "$f" "$O/kernel_trace.csv"
python scripts/trace_gaps.py "$O/kernel_trace.csv" 10 > "$O/gaps.txt" && tail -1 "$O/gaps.txt"
rm -rf "$O/prof"
echo done
