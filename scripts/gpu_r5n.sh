#!/bin/bash
# Round 5: A/B of the weight-gradient kernels at P = 1M (mlp_ablate.py under rocprofv3): k_mlp_wgrad_dma with eight
# waves (4 x 2 blocks) and sixteen (2 x 2), k_mlp_wgrad (GSD_WGRAD_DMA=0), and ablation builds of the eight-wave kernel:
# without MFMAs (GSD_ABLATE=16), without the copies after the first pair (4096), with the hi plane only (8192).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5n}; O="gpurun_out/$OUT"; mkdir -p "$O"
L=gaussian-splatting_deformable_amd
run() {   # name, then env assignments
  local name=$1; shift
  env "$@" timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$name" -o run -- \
      python scripts/mlp_ablate.py --reps 5 > "$O/ablate_$name.log" 2>&1 || { tail -20 "$O/ablate_$name.log"; return 1; }
  local f; f=$(find "$O/prof_$name" -name '*kernel_stats.csv' | head -1)
  echo "== $name"; grep -i "wgrad" "$f" | cut -d, -f1-8
}
run dma8 GSD_WGRAD_DMA=8 && run dma16 GSD_WGRAD_DMA=16 && run old GSD_WGRAD_DMA=0 && \
run abl16 GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L/build_abl16/libgsd_hip.so && \
run abl4096 GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L/build_abl4096/libgsd_hip.so && \
run abl8192 GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L/build_abl8192/libgsd_hip.so && \
run dma8b GSD_WGRAD_DMA=8 && echo all-done
