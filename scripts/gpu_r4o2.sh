#!/bin/bash
# Round 4: kernel statistics of the driver's bench command at HEAD (rocprofv3 --kernel-trace --stats), with the
# bench line of the same run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r4o2}"; mkdir -p "$O"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py \
    > "$O/bench_prof.log" 2>&1 || { tail -20 "$O/bench_prof.log"; exit 1; }
find "$O/prof" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$O/bench_kernel_stats.csv"
grep '^{"metric"' "$O/bench_prof.log" | tail -1 | cut -c1-200
python3 scripts/kstats.py --match render "$O/bench_kernel_stats.csv"
