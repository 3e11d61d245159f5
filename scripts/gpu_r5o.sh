#!/bin/bash
# Round 5: k_mlp_wgrad_dma variants at P = 1M (mlp_ablate.py under rocprofv3): GSD_WGRAD_DMA = 8 (eight waves of
# 4 x 2 blocks, product-major MFMA order), 80 (the same block by block), 4 (four waves of 4 x 4), 16 (sixteen of
# 2 x 2), 0 (k_mlp_wgrad).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5o}; O="gpurun_out/$OUT"; mkdir -p "$O"
run() {   # name, then env assignments
  local name=$1; shift
  env "$@" timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$name" -o run -- \
      python scripts/mlp_ablate.py --reps 5 > "$O/ablate_$name.log" 2>&1 || { tail -20 "$O/ablate_$name.log"; return 1; }
  local f; f=$(find "$O/prof_$name" -name '*kernel_stats.csv' | head -1)
  echo "== $name"; grep -i "wgrad" "$f" | cut -d, -f1-4
}
run dma8 GSD_WGRAD_DMA=8 && run dma80 GSD_WGRAD_DMA=80 && run dma4 GSD_WGRAD_DMA=4 && run round1 GSD_WGRAD_DMA=0 GSD_WGRAD_ROUND1=1 && \
run old GSD_WGRAD_DMA=0 && run dma16 GSD_WGRAD_DMA=16 && run round1b GSD_WGRAD_DMA=0 GSD_WGRAD_ROUND1=1 && echo all-done
