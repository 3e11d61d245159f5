#!/bin/bash
# Round 5: k_tile_sort with a 256-key register network for buckets of <= 256 keys (one key per lane, 36 passes)
# instead of the 512-key one -- the binning parity tests, then prof_render.py --timing at cfg4 against build_base/
# (HEAD before the change), A/B/A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5ae}; O="gpurun_out/$OUT"; mkdir -p "$O"
L=gaussian-splatting_deformable_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread \
    > "$O/tests.txt" 2>&1 || { tail -30 "$O/tests.txt"; exit 1; }
tail -2 "$O/tests.txt"
for rep in 1 2; do
  for v in build build_base; do
    GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L/$v/libgsd_hip.so timeout -k 10 300 python scripts/prof_render.py --iters 30 --timing \
        > "$O/prof_${v}_$rep.log" 2>&1 || { tail -20 "$O/prof_${v}_$rep.log"; exit 1; }
    echo "== $v $rep"; grep "sort\|scatter\|hist" "$O/prof_${v}_$rep.log"
  done
done
echo all-done
