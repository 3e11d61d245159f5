#!/bin/bash
# Round 5: k_render_bwd at six waves per SIMD (build_w6/, -DGSD_BWD_GROUPS_WAVES=6: 80 VGPRs, 13 spilled) against
# the tree's five: prof_render.py --timing at cfg4, A/B/A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5ab}; O="gpurun_out/$OUT"; mkdir -p "$O"
L=gaussian-splatting_deformable_amd
for rep in 1 2; do
  for v in build build_w6; do
    GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L/$v/libgsd_hip.so timeout -k 10 300 python scripts/prof_render.py --iters 30 --timing \
        > "$O/prof_${v}_$rep.log" 2>&1 || { tail -20 "$O/prof_${v}_$rep.log"; exit 1; }
    echo "== $v $rep"; grep "render_bwd" "$O/prof_${v}_$rep.log"
  done
done
echo all-done
