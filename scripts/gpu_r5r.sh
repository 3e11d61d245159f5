#!/bin/bash
# Round 5: the deformation-network GPU tests with the one-round 256 x 256 weight gradient as the default (and its
# large-P test), then the training call's kernel statistics at P = 1M.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5r}; O="gpurun_out/$OUT"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py -x -v -m gpu --timeout 400 --timeout-method thread \
    > "$O/gpu_mlp_tests.txt" 2>&1 || { tail -40 "$O/gpu_mlp_tests.txt"; exit 1; }
tail -3 "$O/gpu_mlp_tests.txt"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
    python scripts/mlp_ablate.py --reps 5 > "$O/ablate.log" 2>&1 || { tail -20 "$O/ablate.log"; exit 1; }
f=$(find "$O/prof" -name '*kernel_stats.csv' | head -1); cp "$f" "$O/kernel_stats.csv"
echo all-done
