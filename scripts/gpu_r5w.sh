#!/bin/bash
# Round 5: k_mlp_wgrad (the 256 x 256 weight gradient, one round of chunks) with and without its MFMAs
# (GSD_ABLATE=16, timing only): how much of its time the staging (loads + split + LDS writes) alone takes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5w}; O="gpurun_out/$OUT"; mkdir -p "$O"
L=gaussian-splatting_deformable_amd
for v in build build_abl16; do
  GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L/$v/libgsd_hip.so timeout -k 10 240 rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$O/prof_$v" -o run -- python scripts/mlp_ablate.py --reps 5 > "$O/ablate_$v.log" 2>&1 \
      || { tail -20 "$O/ablate_$v.log"; exit 1; }
  f=$(find "$O/prof_$v" -name '*kernel_stats.csv' | head -1)
  echo "== $v"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'wgrad' in r['Name']: print(f\"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>3}  {r['Name'][:60]}\")"
done
echo all-done
