#!/bin/bash
# bench.py on every BASELINE configuration (1-5) on one GPU, each step its own time limit; lines into
# gpurun_out/$OUT/bench_cfgN.json.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-cfgs}"; mkdir -p "$O"
for c in ${CFGS:-1 2 3 4 5}; do
  timeout -k 10 300 python3 bench.py --config $c --steps ${STEPS:-50} --warmup ${WARMUP:-10} > "$O/bench_cfg$c.log" 2>&1 || { echo "cfg$c failed"; tail -20 "$O/bench_cfg$c.log"; exit 1; }
  tail -1 "$O/bench_cfg$c.log" > "$O/bench_cfg$c.json"
  python3 -c "import json; d=json.load(open('$O/bench_cfg$c.json')); r=d['roofline'] or {}; print('cfg$c', d['value'], d['ms_per_step'], d['fwd_bwd_ms_per_view'], r.get('kernel'), r.get('bound'), r.get('frac'), r.get('traffic'))"
done
echo configs-done
