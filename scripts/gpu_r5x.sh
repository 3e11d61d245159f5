#!/bin/bash
# Round 5: k_mlp_wgrad_split (LDS-DMA raw rows, each element split once) -- the deformation-network GPU tests, then the
# training call's kernel statistics with it and with GSD_WGRAD_SPLIT=0 (k_mlp_wgrad), A/B/A.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5x}; O="gpurun_out/$OUT"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_mlp.py -x -v -m gpu --timeout 400 --timeout-method thread \
    > "$O/gpu_mlp_tests.txt" 2>&1 || { tail -40 "$O/gpu_mlp_tests.txt"; exit 1; }
tail -2 "$O/gpu_mlp_tests.txt"
i=0
for v in 1 0 1; do
  i=$((i + 1))
  GSD_WGRAD_SPLIT=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$i" -o run -- \
      python scripts/mlp_ablate.py --reps 5 > "$O/ablate_$i.log" 2>&1 || { tail -20 "$O/ablate_$i.log"; exit 1; }
  f=$(find "$O/prof_$i" -name '*kernel_stats.csv' | head -1)
  echo "== GSD_WGRAD_SPLIT=$v"; python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'wgrad' in r['Name'] or 'chain' in r['Name'] or 'fused' in r['Name']: print(f\"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>3}  {r['Name'][:60]}\")"
done
echo all-done
