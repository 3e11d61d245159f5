#!/bin/bash
# Round 5: k_ssim_fwd's horizontal pass with two output columns per thread from b128 LDS reads (build/) against the
# 8-B-per-tap pass (build_base/, -DGSD_SSIM_FWD_SCALAR_H): prof_loss.py under rocprofv3, A/B x3, then the loss tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5ax}; O="gpurun_out/$OUT"; mkdir -p "$O"
L=gaussian-splatting_deformable_amd
for rep in 1 2 3; do
  for v in build_base build; do
    GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L/$v/libgsd_hip.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$O/prof_${v}_$rep" -o run -- python scripts/prof_loss.py --iters 100 > "$O/loss_${v}_$rep.log" 2>&1 \
        || { tail -20 "$O/loss_${v}_$rep.log"; exit 1; }
    f=$(find "$O/prof_${v}_$rep" -name '*kernel_stats.csv' | head -1)
    echo "== $v $rep"; python3 -c "import csv,sys; [print(r[\"Name\"][:24], r[\"Calls\"], r[\"AverageNs\"]) for r in csv.DictReader(open(sys.argv[1])) if \"ssim\" in r[\"Name\"]]" "$f"
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -x -q -m gpu -k "ssim or loss" --timeout 300 --timeout-method thread > "$O/tests.txt" 2>&1 || { tail -30 "$O/tests.txt"; exit 1; }
tail -2 "$O/tests.txt"
echo all-done
