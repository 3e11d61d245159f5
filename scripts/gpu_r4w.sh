#!/bin/bash
# Round 4 final pass, part 2: PMC passes over the cfg4 render step (FETCH_SIZE; WRITE_SIZE; the SQ group) and every
# BASELINE configuration's bench line; then the MLP tests + kernel statistics (gpu_r4l.sh) and the MLP-live bench
# line with its kernel statistics.  Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r4w}"; mkdir -p "$O"
PMC_OUT="$O/pmc" PMC_PASSES="FETCH_SIZE;WRITE_SIZE;SQ_INSTS_VALU GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_LDS" \
    bash scripts/gpu_pmc.sh || exit 1
OUT="${OUT:-r4w}/cfgs" STEPS=20 WARMUP=5 bash scripts/gpu_configs.sh || exit 1
OUT="${OUT:-r4w}/mlp" bash scripts/gpu_r4l.sh || exit 1
timeout -k 10 300 python bench.py --with-mlp --steps 10 --warmup 3 --cpu-baseline off > "$O/bench_mlp.log" 2>&1 \
    || { tail -20 "$O/bench_mlp.log"; exit 1; }
tail -1 "$O/bench_mlp.log" | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_mlp" -o run -- python3 bench.py \
    --with-mlp --steps 5 --warmup 2 --cpu-baseline off > "$O/bench_mlp_prof.log" 2>&1 || { tail -20 "$O/bench_mlp_prof.log"; exit 1; }
find "$O/prof_mlp" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$O/bench_mlp_kernel_stats.csv"
echo all-done
