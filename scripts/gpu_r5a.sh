#!/bin/bash
# Round 5 baseline at HEAD: the driver's bench command and the rasterizer-only kernel times (cfg4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r5a}"; mkdir -p "$O"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver.log" 2>&1 || { tail -20 "$O/bench_driver.log"; exit 1; }
tail -1 "$O/bench_driver.log" | cut -c1-300
timeout -k 10 300 python scripts/prof_render.py --iters 30 --timing > "$O/prof_render.log" 2>&1 || { tail -20 "$O/prof_render.log"; exit 1; }
cat "$O/prof_render.log" | grep -v amdgpu.ids
echo done
