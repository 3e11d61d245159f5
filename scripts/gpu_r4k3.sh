#!/bin/bash
# Round 4: k_ssim_fwd at 512 threads (two output rows per thread, 54 VGPRs, six waves per SIMD) against 256 (four
# rows, 146 VGPRs, three) -- the loss GPU tests with each library, then bench kernel statistics A/B/A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r4k3}"; mkdir -p "$O"
for lib in build build_ssim512; do
  GSD_HIP_LIB=$PWD/gaussian-splatting_deformable_amd/$lib/libgsd_hip.so timeout -k 10 300 python -u -m pytest -x -q \
      --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_configs.py \
      > "$O/tests_$lib.log" 2>&1 || { tail -40 "$O/tests_$lib.log"; exit 1; }
  echo "$lib: $(tail -1 "$O/tests_$lib.log")"
done
i=0
for lib in build build_ssim512 build build_ssim512; do
  i=$((i+1))
  GSD_HIP_LIB=$PWD/gaussian-splatting_deformable_amd/$lib/libgsd_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$O/p$i" -o run -- python3 bench.py --steps 20 --warmup 5 --cpu-baseline off \
      > "$O/bench$i.log" 2>&1 || { tail -20 "$O/bench$i.log"; exit 1; }
  find "$O/p$i" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$O/stats_$i.csv"
  echo "$lib"; python3 scripts/kstats.py --match "k_ssim" "$O/stats_$i.csv"
done
