#!/bin/bash
# Round 5 final check at HEAD: the whole -m gpu suite, smoke(), the driver's bench command with its rocprofv3 kernel
# statistics (gpu_full.sh); no PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5final}; O="gpurun_out/$OUT"; mkdir -p "$O"
export GSD_PARITY_REPORT="$O/parity_flips.jsonl"
PROF=1 OUT=$OUT bash scripts/gpu_full.sh || exit 1
echo all-done
