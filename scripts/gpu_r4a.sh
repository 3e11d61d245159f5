#!/bin/bash
# Round-4 check: the -m gpu tests (parity flip counts appended to parity_flips.jsonl), then per-kernel times of
# prof_render.py (cfg 4, 30 fwd+bwd passes).  TESTS overrides the test selection, OUT the output directory.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r4a}"; mkdir -p "$O"
export GSD_PARITY_REPORT="$O/parity_flips.jsonl"
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > "$O/gpu_tests.log" 2>&1 || { tail -40 "$O/gpu_tests.log"; exit 1; }
tail -3 "$O/gpu_tests.log"
timeout -k 10 200 python scripts/prof_render.py --iters 30 --timing > "$O/quick.log" 2>&1 && grep -v amdgpu.ids "$O/quick.log"
