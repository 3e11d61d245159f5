#!/bin/bash
# Round 5 final check at HEAD: the whole -m gpu suite, smoke(), the driver's bench command with its rocprofv3 kernel
# statistics (gpu_full.sh); with COUNT=1 the useful-work counters; no PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5final}; O="gpurun_out/$OUT"; mkdir -p "$O"
export GSD_PARITY_REPORT="$O/parity_flips.jsonl"
PROF=1 OUT=$OUT bash scripts/gpu_full.sh || exit 1
if [ -n "$COUNT" ]; then  # the useful-work counters (build_count/, -DGSD_COUNT_WORK) at cfg4
  GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB=gaussian-splatting_deformable_amd/build_count/libgsd_hip.so timeout -k 10 200 \
      python scripts/count_work.py --config 4 --out "$O/work_counts_cfg4.json" > "$O/count.log" 2>&1 || { tail -20 "$O/count.log"; exit 1; }
  cat "$O/work_counts_cfg4.json"
fi
echo all-done
