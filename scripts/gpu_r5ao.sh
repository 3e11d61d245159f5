#!/bin/bash
# Round 5: the 256 x 256 weight gradient staging with two threads per row (every wave stages eight Gaussians of a
# row; build_wh/) against HEAD (build_base/, half the waves stage whole 16-Gaussian segments): mlp_ablate.py under
# rocprofv3, A/B/A/B, then the network tests on the variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5ao}; O="gpurun_out/$OUT"; mkdir -p "$O"
L=gaussian-splatting_deformable_amd
for rep in 1 2; do
  for v in build_base build_wh; do
    GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L/$v/libgsd_hip.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$O/prof_${v}_$rep" -o run -- python scripts/mlp_ablate.py --reps 5 > "$O/ablate_${v}_$rep.log" 2>&1 \
        || { tail -20 "$O/ablate_${v}_$rep.log"; exit 1; }
    f=$(find "$O/prof_${v}_$rep" -name '*kernel_stats.csv' | head -1)
    echo "== $v $rep"; grep -i "wgrad<8, 8" "$f" | cut -d, -f1-4
  done
done
GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L/build_wh/libgsd_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py -x -q \
    -m gpu --timeout 300 --timeout-method thread > "$O/tests_wh.txt" 2>&1 || { tail -30 "$O/tests_wh.txt"; exit 1; }
tail -2 "$O/tests_wh.txt"
echo all-done
