#!/bin/bash
# Round 4: the backward dX chain -- the MLP GPU tests, kernel statistics of scripts/mlp_ablate.py with the product
# library and with the register-copy forward variant (build_abl2048).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=r4o bash scripts/gpu_r4l.sh && VARIANTS="2048" OUT=r4o bash scripts/gpu_r4k.sh
