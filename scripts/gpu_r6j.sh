#!/bin/bash
# Round 6: the 20-step bench's first-step transient -- per-step device and host times for the driver's command
# (A), with no restore between the warmup and the timed steps (B), with 60 warmup steps (C) and on the drop-in
# step (D).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
OUT=${OUT:-r6j}; O="gpurun_out/$OUT"; mkdir -p "$O"
run() {  # name, env..., -- bench args
  local name=$1; shift
  env GSD_BENCH_STEP_TIMES=1 "$@" > "$O/$name.log" 2>&1 || { tail -20 "$O/$name.log"; return 1; }
  echo "== $name"; grep -E "^(step|host) ms" "$O/$name.log"
  grep '^{"metric"' "$O/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['num_rendered_timed_first'], d['config']['num_rendered_timed_last'])"
}
run A timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off &&
run B GSD_BENCH_RESTORE_FIRST=1 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off &&
run C timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 60 --cpu-baseline off &&
run D GSD_TRAIN_STEP=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off &&
echo all-done
