#!/bin/bash
# Round 4: the MLP tests + kernel statistics (gpu_r4l.sh), then the MLP-live bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r4t}"; mkdir -p "$O"
OUT="${OUT:-r4t}/mlp" bash scripts/gpu_r4l.sh || exit 1
timeout -k 10 300 python bench.py --with-mlp --steps 10 --warmup 3 --cpu-baseline off > "$O/bench_mlp.log" 2>&1 \
    || { tail -20 "$O/bench_mlp.log"; exit 1; }
tail -1 "$O/bench_mlp.log" | cut -c1-200
