#!/bin/bash
# Round 4: the forward's six-slot ring (one wait + barrier per two k-steps) -- the MLP tests, then
# scripts/mlp_ablate.py kernel statistics A/B/A against the four-slot ring (build_ring4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r4n2}"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mlp.py \
    > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
i=0
for lib in build build_ring4 build; do
  i=$((i+1))
  GSD_HIP_LIB=$PWD/gaussian-splatting_deformable_amd/$lib/libgsd_hip.so timeout -k 10 180 rocprofv3 --kernel-trace \
      --stats --output-format csv -d "$O/p$i" -o run -- python3 scripts/mlp_ablate.py --reps 5 > "$O/abl$i.log" 2>&1 \
      || { tail -20 "$O/abl$i.log"; exit 1; }
  find "$O/p$i" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$O/stats_$i.csv"
  python3 scripts/kstats.py --match fwd_fused "$O/stats_$i.csv"
done
