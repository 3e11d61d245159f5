#!/bin/bash
# Round 4: the MLP-live bench line under rocprofv3 --kernel-trace --stats at HEAD (the line and the kernel statistics
# from the same run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r4l2}"; mkdir -p "$O"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py \
    --with-mlp --steps 10 --warmup 3 --cpu-baseline off > "$O/bench_prof.log" 2>&1 || { tail -20 "$O/bench_prof.log"; exit 1; }
find "$O/prof" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$O/bench_mlp_kernel_stats.csv"
grep '^{"metric"' "$O/bench_prof.log" | tail -1 | cut -c1-160
