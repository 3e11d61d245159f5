#!/bin/bash
# Round 5: the 256 x 256 weight gradient with half of each SIMD's waves multiplying before staging (build_ho/,
# -DGSD_WGRAD_HALF_ORDER) against HEAD (build/): mlp_ablate.py under rocprofv3, A/B x2, then the network tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5ar}; O="gpurun_out/$OUT"; mkdir -p "$O"
L=gaussian-splatting_deformable_amd
for rep in 1 2 3; do
  for v in build build_ho; do
    GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L/$v/libgsd_hip.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$O/prof_${v}_$rep" -o run -- python scripts/mlp_ablate.py --reps 5 > "$O/ablate_${v}_$rep.log" 2>&1 \
        || { tail -20 "$O/ablate_${v}_$rep.log"; exit 1; }
    f=$(find "$O/prof_${v}_$rep" -name '*kernel_stats.csv' | head -1)
    echo "== $v $rep"; python3 -c "import csv,sys; [print(r[\"Name\"][:40], r[\"Calls\"], r[\"AverageNs\"]) for r in csv.DictReader(open(sys.argv[1])) if \"k_mlp_wgrad<\" in r[\"Name\"]]" "$f"
  done
done
GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L/build_ho/libgsd_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py -x -q \
    -m gpu --timeout 300 --timeout-method thread > "$O/tests_ho.txt" 2>&1 || { tail -30 "$O/tests_ho.txt"; exit 1; }
tail -2 "$O/tests_ho.txt"
echo all-done
