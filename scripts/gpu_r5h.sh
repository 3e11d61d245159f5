#!/bin/bash
# Round 5: parity statistics at HEAD (flip margins, final_T relative deviation) from the full parity and configuration
# tests, then the driver's bench command and its rocprofv3 kernel statistics.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r5h}"; mkdir -p "$O"
export GSD_PARITY_REPORT="$O/parity_flips.jsonl"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_render_modes.py -x -q \
    -p no:cacheprovider --timeout 200 --timeout-method thread > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver.log" 2>&1 || { tail -20 "$O/bench_driver.log"; exit 1; }
tail -1 "$O/bench_driver.log" | cut -c1-300
echo done
