#!/bin/bash
# Round 5: the MLP-live bench line (bench.py --with-mlp) and its rocprofv3 kernel statistics at HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5mlp}; O="gpurun_out/$OUT"; mkdir -p "$O"
timeout -k 10 300 python bench.py --with-mlp --steps 10 --warmup 3 --cpu-baseline off > "$O/bench_mlp.log" 2>&1 \
    || { tail -20 "$O/bench_mlp.log"; exit 1; }
tail -1 "$O/bench_mlp.log" | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_mlp" -o run -- python3 bench.py \
    --with-mlp --steps 5 --warmup 2 --cpu-baseline off > "$O/bench_mlp_prof.log" 2>&1 || { tail -20 "$O/bench_mlp_prof.log"; exit 1; }
find "$O/prof_mlp" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$O/bench_mlp_kernel_stats.csv"
echo all-done
