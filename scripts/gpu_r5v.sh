#!/bin/bash
# Round 5: where k_render_bwd's time goes -- prof_render.py --timing (cfg4) against timing-only builds
# (-DGSD_BWD_ABLATE: 1 no phase 2, 2 no LDS accumulation, 4 no global flush, 8 no walk), the product build first and
# last.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5v}; O="gpurun_out/$OUT"; mkdir -p "$O"
L=gaussian-splatting_deformable_amd
for v in build build_bwdabl1 build_bwdabl2 build_bwdabl4 build_bwdabl8 build; do
  GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L/$v/libgsd_hip.so timeout -k 10 300 python scripts/prof_render.py --iters 30 --timing \
      > "$O/prof_$v.log" 2>&1 || { tail -20 "$O/prof_$v.log"; exit 1; }
  echo "== $v"; grep "render_bwd\|render_fwd" "$O/prof_$v.log"
done
echo all-done
