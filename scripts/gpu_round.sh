#!/bin/bash
# One GPU-box pass at HEAD: scripts/gpu_full.sh (the -m gpu tests, smoke(), the driver's bench command and its
# rocprofv3 kernel-trace summary), then -- with PMC=1 -- the three PMC passes (FETCH_SIZE; WRITE_SIZE; the SQ
# VALU / LDS group) over scripts/prof_render.py for configurations 4 and 5, each into gpurun_out/$OUT/pmc_cfgN.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
OUT="${OUT:-round}"
if [ -z "$SKIP_FULL" ]; then OUT="$OUT" bash scripts/gpu_full.sh || exit 1; fi
if [ -n "$PMC" ]; then
  for c in ${PMC_CFGS:-4 5}; do
    PMC_OUT="gpurun_out/$OUT/pmc_cfg$c" PROF_ARGS="--config $c --iters 3" \
    PMC_PASSES="FETCH_SIZE;WRITE_SIZE;GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES" \
      bash scripts/gpu_pmc.sh || exit 1
  done
fi
echo round-done
