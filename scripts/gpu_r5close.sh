#!/bin/bash
# Round 5 closing pass at the round's last kernels: the PMC passes of the render step at cfg4 and cfg5 (bench.py's
# roofline blocks read them), then every BASELINE configuration's bench line and the MLP-live line (gpu_r5q.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5close}; O="gpurun_out/$OUT"; mkdir -p "$O"
P="FETCH_SIZE;WRITE_SIZE;GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES"
PMC_OUT="$O/pmc_cfg4" PROF_ARGS="--config 4 --iters 3" PMC_PASSES="$P" bash scripts/gpu_pmc.sh || exit 1
PMC_OUT="$O/pmc_cfg5" PROF_ARGS="--config 5 --iters 3" PMC_PASSES="$P" bash scripts/gpu_pmc.sh || exit 1
[ -n "$PMC_ONLY" ] && { echo all-done; exit 0; }
OUT="$OUT/q" bash scripts/gpu_r5q.sh || exit 1
echo all-done
