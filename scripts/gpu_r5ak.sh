#!/bin/bash
# Round 5: both render kernels without register spills (build_ns/: the forward's compaction one slot at a time, the backward's flush constants rebuilt from the image size) against HEAD (build_base/):
# prof_render.py --timing at cfg4, A/B/A/B, then the parity tests on the variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5ak}; O="gpurun_out/$OUT"; mkdir -p "$O"
L=gaussian-splatting_deformable_amd
for rep in 1 2; do
  for v in build_base build_ns; do
    GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L/$v/libgsd_hip.so timeout -k 10 300 python scripts/prof_render.py --iters 30 --timing \
        > "$O/prof_${v}_$rep.log" 2>&1 || { tail -20 "$O/prof_${v}_$rep.log"; exit 1; }
    echo "== $v $rep"; grep "render_bwd\|render_fwd" "$O/prof_${v}_$rep.log"
  done
done
GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L/build_ns/libgsd_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_render_modes.py tests/test_gpu_configs.py -x -q \
    -m gpu --timeout 300 --timeout-method thread > "$O/tests_ns.txt" 2>&1 || { tail -30 "$O/tests_ns.txt"; exit 1; }
tail -2 "$O/tests_ns.txt"
GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=$L/build_ns/libgsd_hip.so PMC_OUT="$O/pmc_cfg4" PROF_ARGS="--config 4 --iters 3" \
  PMC_PASSES="FETCH_SIZE;WRITE_SIZE" bash scripts/gpu_pmc.sh || exit 1
echo all-done
