#!/bin/bash
# Round 4: kernel statistics of the MLP-live bench step (bench.py --with-mlp) under rocprofv3 --kernel-trace --stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r4i}"; mkdir -p "$O"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --gpus 1 \
    --steps 10 --warmup 3 --with-mlp --cpu-baseline off > "$O/bench_prof.log" 2>&1 || { tail -20 "$O/bench_prof.log"; exit 1; }
find "$O/prof" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$O/kernel_stats.csv"
tail -1 "$O/bench_prof.log" | cut -c1-200
