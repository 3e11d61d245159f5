#!/bin/bash
# Round 5: run-to-run spread of the headline on one box -- the driver's bench command five times back to back.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r5aa}; O="gpurun_out/$OUT"; mkdir -p "$O"
for i in 1 2 3 4 5; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off > "$O/bench_$i.log" 2>&1 \
      || { tail -20 "$O/bench_$i.log"; exit 1; }
  tail -1 "$O/bench_$i.log" > "$O/bench_$i.json"
  python3 -c "import json; d=json.load(open('$O/bench_$i.json')); print($i, d['value'], d['ms_per_step'], d['fwd_bwd_ms_per_view'], d['kernels_ms']['render_bwd'], d['kernels_ms']['render_fwd'])"
done
echo all-done
