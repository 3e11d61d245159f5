#!/bin/bash
# Round 5: the per-group backward with double LDS accumulators (ds_add_f64) and 128-record batches -- backward
# parity with it, A/B render_bwd times against the quadrant kernel, and its work counts.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r5k}"; mkdir -p "$O"
L=gaussian-splatting_deformable_amd
GSD_HIP_LIB=$L/build_groups/libgsd_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py \
    -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "backward or config or opacities" > "$O/tests.log" 2>&1 \
    || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
for rep in 1 2; do
  for v in build build_groups build_groups4; do
    GSD_HIP_LIB=$L/$v/libgsd_hip.so timeout -k 10 200 python scripts/prof_render.py --iters 30 --timing \
        > "$O/prof_${v}_$rep.log" 2>&1 || { tail -20 "$O/prof_${v}_$rep.log"; exit 1; }
    echo "== $v $rep: $(grep render_bwd "$O/prof_${v}_$rep.log")"
  done
done
GSD_HIP_LIB=$L/build_count/libgsd_hip.so timeout -k 10 200 python scripts/count_work.py --config 4 --out "$O/work_counts_cfg4.json" \
    > "$O/count.log" 2>&1 || { tail -20 "$O/count.log"; exit 1; }
grep -A3 render_bwd "$O/work_counts_cfg4.json"
echo done
