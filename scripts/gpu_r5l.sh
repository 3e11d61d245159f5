#!/bin/bash
# Round 5 check at HEAD with the per-group backward as the default: the whole -m gpu suite, smoke(), the driver's
# bench command, its rocprofv3 kernel statistics, the useful-work counts (cfg4, cfg5) and the PMC passes of the
# render kernels at cfg4 (FETCH_SIZE; WRITE_SIZE; the SQ VALU / LDS group) for bench.py's roofline block.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5l}; O="gpurun_out/$OUT"; mkdir -p "$O"
export GSD_PARITY_REPORT="$O/parity_flips.jsonl"
PROF=1 OUT=$OUT bash scripts/gpu_full.sh || exit 1
L=gaussian-splatting_deformable_amd
for c in 4 5; do
  GSD_HIP_LIB=$L/build_count/libgsd_hip.so timeout -k 10 200 python scripts/count_work.py --config $c \
      --out "$O/work_counts_cfg$c.json" > "$O/count$c.log" 2>&1 || { tail -20 "$O/count$c.log"; exit 1; }
done
PMC_OUT="$O/pmc_cfg4" PROF_ARGS="--config 4 --iters 3" \
  PMC_PASSES="FETCH_SIZE;WRITE_SIZE;GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_WAVES SQ_WAVE_CYCLES" \
  bash scripts/gpu_pmc.sh || exit 1
echo all-done
