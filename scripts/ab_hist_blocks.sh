#!/bin/bash
# Binning granularity sweep: per-kernel device times of scripts/prof_render.py (cfg 4) with GSD_HIST_BLOCKS
# Gaussian chunks per view (the tile histogram / scatter workgroups; default kHistTargetBlocks = 512).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out/hist
for rep in 1 2; do
  for b in 512 256 1024 2048; do
    GSD_HIST_BLOCKS=$b timeout -k 10 120 python scripts/prof_render.py --config 4 --iters 30 --timing \
        > gpurun_out/hist/b${b}_$rep.log 2>&1 || { tail -5 gpurun_out/hist/b${b}_$rep.log; exit 1; }
    echo "== blocks $b rep $rep"; grep -v amdgpu.ids gpurun_out/hist/b${b}_$rep.log | tail -4
  done
done
