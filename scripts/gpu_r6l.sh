#!/bin/bash
# Round 6: k_mlp_fwd_fused16 + k_mlp_bwd_chain16 (16 Gaussians per wave, two waves per SIMD) -- the MLP GPU tests over the
# kernel pairs, the A/B at 1M Gaussians, then the bench's first-step transient runs (scripts/gpu_r6j.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r6l}; O="gpurun_out/$OUT"; mkdir -p "$O"; export GSD_TEST_MLP16=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_mlp.py -x -v --timeout 120 --timeout-method thread -m gpu \
    > "$O/tests_mlp.log" 2>&1 || { tail -40 "$O/tests_mlp.log"; exit 1; }
tail -3 "$O/tests_mlp.log"
timeout -k 10 300 python -u scripts/mlp_fwd_ab.py --P 1000000 --reps 3 > "$O/mlp_fwd_ab.json" 2> "$O/mlp_fwd_ab.err" \
    || { tail -20 "$O/mlp_fwd_ab.err"; exit 1; }
cat "$O/mlp_fwd_ab.json"
OUT=$OUT/bench bash scripts/gpu_r6j.sh
