#!/bin/bash
# Round 4: the driver's bench command under rocprofv3 --kernel-trace --stats (the kernel statistics the bench
# line's kernels_ms / roofline are checked against), then the plain bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r4h}"; mkdir -p "$O"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --gpus 1 \
    --steps 20 --warmup 5 --cpu-baseline off > "$O/bench_prof.log" 2>&1 || { tail -20 "$O/bench_prof.log"; exit 1; }
find "$O/prof" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$O/kernel_stats.csv"
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-300
