#!/bin/bash
# Round 4: SSIM backward with each adjoint map aliased by its horizontal sums (21 KB of LDS, seven waves per SIMD) -- the parity / render-mode / training GPU tests, then
# bench kernel statistics with the product library and with the previous loss kernels (build_lossold), A/B/A.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r4v}"; mkdir -p "$O"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_configs.py \
    tests/test_gpu_render_modes.py > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
i=0
for lib in build build_lossold build; do
  i=$((i+1))
  GSD_HIP_LIB=$PWD/gaussian-splatting_deformable_amd/$lib/libgsd_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$O/p$i" -o run -- python3 bench.py --steps 20 --warmup 5 --cpu-baseline off \
      > "$O/bench$i.log" 2>&1 || { tail -20 "$O/bench$i.log"; exit 1; }
  find "$O/p$i" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$O/stats_$i.csv"
  python3 scripts/kstats.py --match "k_ssim" "$O/stats_$i.csv"
  tail -1 "$O/bench$i.log" | cut -c1-120
done
