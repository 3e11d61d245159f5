#!/bin/bash
# Round 6: the driver's 20-step bench command with per-step device times (GSD_BENCH_STEP_TIMES) after the one-call
# step's no-rebuild fix, twice, and the 100-step line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r6i}; O="gpurun_out/$OUT"; mkdir -p "$O"
for rep in 1 2; do
  GSD_BENCH_STEP_TIMES=1 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off > "$O/b20_$rep.log" 2>&1 \
      || { tail -20 "$O/b20_$rep.log"; exit 1; }
  grep "step ms" "$O/b20_$rep.log"
  grep '^{"metric"' "$O/b20_$rep.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('20 steps', d['value'], d['ms_per_step'], d['dropin_api_step'])"
done
timeout -k 10 400 python3 bench.py --steps 100 --warmup 10 --cpu-baseline off > "$O/b100.log" 2>&1 || { tail -20 "$O/b100.log"; exit 1; }
grep '^{"metric"' "$O/b100.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('100 steps', d['value'], d['ms_per_step'], d['dropin_api_step'])"
echo all-done
