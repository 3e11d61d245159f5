#!/bin/bash
# Round 5: the forward's walk ended at the longest list of the groups with an unsaturated pixel.  Render parity tests,
# the useful-work counts at cfg4 (-DGSD_COUNT_WORK build), then per-kernel times of the rasterizer (prof_render.py,
# cfg4) alternating the tree's library with build_base/ (HEAD before the change), A/B/A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5u}; O="gpurun_out/$OUT"; mkdir -p "$O"
L=gaussian-splatting_deformable_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_render_modes.py -x -q -m gpu --timeout 300 \
    --timeout-method thread > "$O/tests.txt" 2>&1 || { tail -30 "$O/tests.txt"; exit 1; }
tail -2 "$O/tests.txt"
GSD_HIP_LIB=$L/build_count/libgsd_hip.so timeout -k 10 200 python scripts/count_work.py --config 4 \
    --out "$O/work_counts_cfg4.json" > "$O/count4.log" 2>&1 || { tail -20 "$O/count4.log"; exit 1; }
cat "$O/work_counts_cfg4.json"
for rep in 1 2; do
  for v in cur base; do
    lib=$L/build/libgsd_hip.so; [ $v = base ] && lib=$L/build_base/libgsd_hip.so
    GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$lib timeout -k 10 300 python scripts/prof_render.py --iters 30 --timing \
        > "$O/prof_${v}_$rep.log" 2>&1 || { tail -20 "$O/prof_${v}_$rep.log"; exit 1; }
    echo "== $v $rep"; grep -i "render\|total" "$O/prof_${v}_$rep.log" | head -6
  done
done
echo all-done
