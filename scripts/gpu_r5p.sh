#!/bin/bash
# Round 5 closing pass, part 1: the whole -m gpu suite, smoke(), the driver's bench command with its rocprofv3 kernel
# statistics (gpu_full.sh), and the PMC passes of the render step at cfg4 under the kernels' final names.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5p}; O="gpurun_out/$OUT"; mkdir -p "$O"
export GSD_PARITY_REPORT="$O/parity_flips.jsonl"
PROF=1 OUT=$OUT bash scripts/gpu_full.sh || exit 1
PMC_OUT="$O/pmc_cfg4" PROF_ARGS="--config 4 --iters 3" \
  PMC_PASSES="FETCH_SIZE;WRITE_SIZE;GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES" \
  bash scripts/gpu_pmc.sh || exit 1
echo all-done
