#!/bin/bash
# Round 6: render micro-changes (0.99 clamp from an SGPR, the forward's contributor by list index) -- parity, then
# A/B against HEAD~ (build_ab_base) and the bare-reciprocal variant (build_v1r).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r6c}; O="gpurun_out/$OUT"; mkdir -p "$O"
export GSD_PARITY_REPORT="$O/parity_flips.jsonl"
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_configs.py -k "not densify" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
OUT="$OUT/ab" LIBS="base:gaussian-splatting_deformable_amd/build_ab_base cur:gaussian-splatting_deformable_amd/build v1r:gaussian-splatting_deformable_amd/build_v1r" \
    REPS=3 bash scripts/ab_libs.sh || exit 1
echo all-done
