#!/bin/bash
# Round 4: 16-wave weight-gradient experiment (GSD_WGRAD16=1: 2 x 2 blocks per wave, 4 waves per SIMD) -- the MLP
# tests with it, then scripts/mlp_ablate.py kernel statistics without / with / without.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r4u}"; mkdir -p "$O"
GSD_WGRAD16=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mlp.py \
    > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
i=0
for w in 0 1 0; do
  i=$((i+1))
  GSD_WGRAD16=$w timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/p$i" -o run -- \
      python3 scripts/mlp_ablate.py --reps 5 > "$O/abl$i.log" 2>&1 || { tail -20 "$O/abl$i.log"; exit 1; }
  find "$O/p$i" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$O/stats_$i.csv"
  python3 scripts/kstats.py --match wgrad "$O/stats_$i.csv"
done
