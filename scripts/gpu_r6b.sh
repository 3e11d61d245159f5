#!/bin/bash
# Round 6: per-instruction-form VALU costs (scripts/calib/valu_cost.hip) and the bench step's PMC passes with
# GSD_BENCH_STEP_ONLY=1 (only warmup + timed steps under the counters: every launch is a bench step's).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r6b}; O="gpurun_out/$OUT"; mkdir -p "$O"
timeout -k 10 120 scripts/calib/valu_cost > "$O/valu_cost.txt" 2>&1 || { tail -5 "$O/valu_cost.txt"; exit 1; }
cat "$O/valu_cost.txt"
B1="FETCH_SIZE GRBM_GUI_ACTIVE"
B2="WRITE_SIZE SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
GSD_BENCH_STEP_ONLY=1 PMC_OUT="$O/bench_pmc" PROF_SCRIPT=bench.py PROF_ARGS="--gpus 1 --steps 10 --warmup 3 --cpu-baseline off" \
    PMC_PASSES="$B1;$B2" bash scripts/gpu_pmc.sh || exit 1
echo all-done
