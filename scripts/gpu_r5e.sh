#!/bin/bash
# Round 5: the per-group-list render_bwd -- backward parity tests, A/B kernel times against the quadrant kernel
# (build_quad/, -DGSD_BWD_QUADRANT), and the useful-work counters (build_count/, -DGSD_COUNT_WORK).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r5e}"; mkdir -p "$O"
L=gaussian-splatting_deformable_amd
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -p no:cacheprovider \
    --timeout 200 --timeout-method thread -k "backward_matches" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
for rep in 1 2; do
  for v in build build_quad build_qnoadd build_write; do
    GSD_HIP_LIB=$L/$v/libgsd_hip.so timeout -k 10 200 python scripts/prof_render.py --iters 30 --timing \
        > "$O/prof_${v}_$rep.log" 2>&1 || { tail -20 "$O/prof_${v}_$rep.log"; exit 1; }
    echo "== $v $rep: $(grep render_bwd "$O/prof_${v}_$rep.log")"
  done
done
echo done
