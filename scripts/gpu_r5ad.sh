#!/bin/bash
# Round 5: what the SSIM forward's three adjoint-map stores cost -- prof_loss.py under rocprofv3 with the tree's build
# and a timing-only build that folds the maps into the sum instead of storing them (-DGSD_SSIM_ABL_NOSTORE).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5ad}; O="gpurun_out/$OUT"; mkdir -p "$O"
L=gaussian-splatting_deformable_amd
for v in build build_ssimabl build; do
  GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L/$v/libgsd_hip.so timeout -k 10 240 rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$O/prof_$v" -o run -- python scripts/prof_loss.py --iters 100 > "$O/loss_$v.log" 2>&1 \
      || { tail -20 "$O/loss_$v.log"; exit 1; }
  f=$(find "$O/prof_$v" -name '*kernel_stats.csv' | head -1)
  echo "== $v"; python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'ssim' in r['Name'] or 'loss_sum' in r['Name']: print(f\"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4}  {r['Name'][:50]}\")"
done
echo all-done
