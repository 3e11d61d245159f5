#!/bin/bash
# Round 5: k_scatter_hist with nontemporal key stores (build_nt/, -DGSD_SCATTER_NT) against HEAD (build_base/):
# prof_render.py A/B, then the parity tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5av}; O="gpurun_out/$OUT"; mkdir -p "$O"
L=gaussian-splatting_deformable_amd
for rep in $(seq 1 ${REPS:-2}); do
  for v in build_base build_nt; do
    GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L/$v/libgsd_hip.so timeout -k 10 300 python scripts/prof_render.py --iters ${ITERS:-30} --timing \
        > "$O/prof_${v}_$rep.log" 2>&1 || { tail -20 "$O/prof_${v}_$rep.log"; exit 1; }
    echo "== $v $rep"; grep "scatter\|tile_sort\|render_fwd" "$O/prof_${v}_$rep.log"
  done
done
[ -n "$NOTEST" ] && { echo all-done; exit 0; }
GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L/build_nt/libgsd_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_render_modes.py tests/test_gpu_configs.py -x -q \
    -m gpu --timeout 300 --timeout-method thread > "$O/tests_nt.txt" 2>&1 || { tail -30 "$O/tests_nt.txt"; exit 1; }
tail -2 "$O/tests_nt.txt"
echo all-done
