#!/bin/bash
# Round 5: PMC passes of the render step at cfg5 (2M Gaussians, 4K) with the per-group backward, for bench.py's
# roofline block of that configuration.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5s}; O="gpurun_out/$OUT"; mkdir -p "$O"
PMC_OUT="$O/pmc_cfg5" PROF_ARGS="--config 5 --iters 3" \
  PMC_PASSES="FETCH_SIZE;WRITE_SIZE;GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES" \
  bash scripts/gpu_pmc.sh || exit 1
echo all-done
