#!/bin/bash
# Round 4: what each part of the MLP training kernels costs -- kernel statistics of scripts/mlp_ablate.py (P = 1M)
# with the product library and with each -DGSD_ABLATE=<bit> build (gaussian-splatting_deformable_amd/build_abl<bit>).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r4k}"; mkdir -p "$O"
for v in ${VARIANTS:-0 1 2 4 8 16 64 128}; do
  lib=gaussian-splatting_deformable_amd/build/libgsd_hip.so
  [ "$v" != 0 ] && lib=gaussian-splatting_deformable_amd/build_abl$v/libgsd_hip.so
  GSD_HIP_LIB=$PWD/$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/p$v" -o run -- \
      python3 scripts/mlp_ablate.py --reps 5 > "$O/abl$v.log" 2>&1 || { echo "variant $v failed"; tail -20 "$O/abl$v.log"; exit 1; }
  find "$O/p$v" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$O/stats_$v.csv"
  echo "variant $v: $(tail -1 "$O/abl$v.log")"
done
