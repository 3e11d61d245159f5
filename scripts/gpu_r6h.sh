#!/bin/bash
# Round 6 check at HEAD: the whole -m gpu suite (with the reference alpha mode's strict-bar tests), smoke(), the
# driver's bench command and its rocprofv3 kernel statistics (gpu_full.sh), then the render times of both alpha modes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r6h}; O="gpurun_out/$OUT"; mkdir -p "$O"
export GSD_PARITY_REPORT="$O/parity_flips.jsonl"
PROF=1 OUT=$OUT bash scripts/gpu_full.sh || exit 1
unset GSD_PARITY_REPORT
for m in fast reference; do
  GSD_ALPHA_MODE=$m timeout -k 10 300 python scripts/prof_render.py --iters 30 --timing > "$O/render_$m.log" 2>&1 || exit 1
  echo "$m: $(grep render "$O/render_$m.log" | tr '\n' ' ')"
done
echo all-done
