#!/bin/bash
# Round 4: useful-work counts (GSD_COUNT_WORK build) for configurations 4 and 5, the driver's bench command and
# the MLP-live bench line.  Each GPU step under its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r4e}"; mkdir -p "$O"
for c in ${COUNT_CFGS:-4 5}; do
  GSD_HIP_LIB=gaussian-splatting_deformable_amd/build_count/libgsd_hip.so timeout -k 10 300 \
      python scripts/count_work.py --config $c --out "$O/work_counts_cfg$c.json" > "$O/count_cfg$c.log" 2>&1 \
      || { tail -20 "$O/count_cfg$c.log"; exit 1; }
  tail -1 "$O/count_cfg$c.log"
done
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_cfg4.log" 2>&1 || { tail -20 "$O/bench_cfg4.log"; exit 1; }
tail -1 "$O/bench_cfg4.log" | cut -c1-600
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 3 --with-mlp --cpu-baseline off > "$O/bench_cfg4_mlp.log" 2>&1 \
    || { tail -20 "$O/bench_cfg4_mlp.log"; exit 1; }
tail -1 "$O/bench_cfg4_mlp.log" | cut -c1-600
