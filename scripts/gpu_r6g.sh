#!/bin/bash
# Round 6: the parity cause.  The five configuration parity tests and the parity module on the -DGSD_REFERENCE_ALPHA
# build (alpha = o * expf(power), the oracle's literal expression), flips and T deviations reported; its render times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r6g}; O="gpurun_out/$OUT"; mkdir -p "$O"
L=gaussian-splatting_deformable_amd/build_refalpha/libgsd_hip.so
GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L GSD_PARITY_REPORT="$O/parity_flips_reference_alpha.jsonl" timeout -k 10 600 \
  python -u -m pytest -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_configs.py \
  tests/test_gpu_parity.py -k "full_view or chain or bit_exact or backward_matches" > "$O/refalpha.log" 2>&1
rc=$?; tail -3 "$O/refalpha.log"; [ $rc -gt 1 ] && exit $rc
GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L timeout -k 10 300 python scripts/prof_render.py --iters 30 --timing > "$O/refalpha_timing.log" 2>&1 || exit 1
grep render "$O/refalpha_timing.log"
timeout -k 10 300 python scripts/prof_render.py --iters 30 --timing > "$O/product_timing.log" 2>&1 || exit 1
grep render "$O/product_timing.log"
echo all-done
