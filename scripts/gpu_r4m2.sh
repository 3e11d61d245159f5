#!/bin/bash
# Round 4: configuration 1 (host-bound) with the round-3 tree (.ab/r3, built from 083e46e) and HEAD, alternating:
# is the slower cfg1 line the code or the box?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="$PWD/gpurun_out/${OUT:-r4m2}"; mkdir -p "$O"
for i in 1 2; do
  for t in .ab/r3 .; do
    (cd $t && timeout -k 10 200 python3 bench.py --config 1 --steps 50 --warmup 10 --cpu-baseline off) > "$O/b_$i_$(basename $t).log" 2>&1 \
        || { tail -20 "$O/b_$i_$(basename $t).log"; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('$O/b_$i_$(basename $t).log').read().strip().splitlines()[-1])
print('$t', d['value'], d['ms_per_step'], d.get('fwd_bwd_ms_per_view'), d.get('fwd_bwd_ms_per_view_host_synced'))"
  done
done
