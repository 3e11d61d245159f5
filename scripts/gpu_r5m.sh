#!/bin/bash
# Round 5: the LDS-DMA weight gradient (k_mlp_wgrad_dma, the 256 x 256 layers).  The deformation-network GPU tests,
# then the training call under rocprofv3 with the new kernel and with GSD_WGRAD_DMA=0 (k_mlp_wgrad), A/B/A.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5m}; O="gpurun_out/$OUT"; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py -x -q -m gpu --timeout 240 --timeout-method thread \
    > "$O/gpu_mlp_tests.txt" 2>&1 || { tail -40 "$O/gpu_mlp_tests.txt"; exit 1; }
tail -3 "$O/gpu_mlp_tests.txt"
i=0
for v in 1 0 1; do
  i=$((i + 1))
  GSD_WGRAD_DMA=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$O/prof_$i" -o run -- \
      python scripts/mlp_ablate.py --reps 5 > "$O/ablate_$i.log" 2>&1 || { tail -20 "$O/ablate_$i.log"; exit 1; }
  f=$(find "$O/prof_$i" -name '*kernel_stats.csv' | head -1)
  echo "== GSD_WGRAD_DMA=$v"; grep -i "wgrad\|mlp_fwd_fused\|bwd_chain" "$f" | cut -d, -f1-8
done
echo all-done
