#!/bin/bash
# Round 4 final pass, part 1: the -m gpu suite (parity flip counts into parity_flips.jsonl), the driver's bench
# command, and its kernel statistics under rocprofv3 --kernel-trace --stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r4z}"; mkdir -p "$O"
export GSD_PARITY_REPORT="$O/parity_flips.jsonl"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1 || { tail -40 "$O/gpu_tests.log"; exit 1; }
tail -2 "$O/gpu_tests.log"
timeout -k 10 300 python bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py \
    --steps 20 --warmup 5 --cpu-baseline off > "$O/bench_prof.log" 2>&1 || { tail -20 "$O/bench_prof.log"; exit 1; }
find "$O/prof" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$O/bench_kernel_stats.csv"
echo part1-done
