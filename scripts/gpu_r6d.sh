#!/bin/bash
# Round 6: parity of the bare-reciprocal backward at HEAD (the full -m gpu render suites), the host cost of the step at
# cfg2 (host_split.py, cProfile), and the cfg2 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r6d}; O="gpurun_out/$OUT"; mkdir -p "$O"
export GSD_PARITY_REPORT="$O/parity_flips.jsonl"
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_render_modes.py > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
timeout -k 10 300 python scripts/host_split.py --config 2 --steps 60 > "$O/host_split_cfg2.txt" 2>&1 || { tail -20 "$O/host_split_cfg2.txt"; exit 1; }
tail -15 "$O/host_split_cfg2.txt"
timeout -k 10 300 python scripts/host_profile.py 2 > "$O/host_profile_cfg2.txt" 2>&1 || { tail -20 "$O/host_profile_cfg2.txt"; exit 1; }
head -60 "$O/host_profile_cfg2.txt"
timeout -k 10 300 python bench.py --config 2 --steps 100 --warmup 10 --cpu-baseline off > "$O/bench_cfg2.log" 2>&1 || { tail -20 "$O/bench_cfg2.log"; exit 1; }
grep '^{"metric"' "$O/bench_cfg2.log" | cut -c1-400
echo all-done
