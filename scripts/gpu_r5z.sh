#!/bin/bash
# Round 5: k_preprocess_fwd with the scale / rotation loads issued ahead of the near-plane test (build_hoist/,
# -DGSD_PRE_HOIST=1) against the tree's build: prof_render.py --timing at cfg4, A/B/A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5z}; O="gpurun_out/$OUT"; mkdir -p "$O"
L=gaussian-splatting_deformable_amd
for rep in 1 2; do
  for v in build build_hoist; do
    GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L/$v/libgsd_hip.so timeout -k 10 300 python scripts/prof_render.py --iters 30 --timing \
        > "$O/prof_${v}_$rep.log" 2>&1 || { tail -20 "$O/prof_${v}_$rep.log"; exit 1; }
    echo "== $v $rep"; grep "preprocess\|render_fwd" "$O/prof_${v}_$rep.log"
  done
done
echo all-done
