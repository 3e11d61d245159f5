#!/bin/bash
# GSD_FWD_ZERO_SCRATCH=1 vs 0 on configurations 2 and 3 (host-/launch-bound small steps), alternating on one box.
set -o pipefail
mkdir -p gpurun_out/abc
for rep in 1 2; do
  for c in 2 3; do
    for z in 1 0; do
      GSD_FWD_ZERO_SCRATCH=$z timeout -k 10 200 python3 bench.py --config $c --steps 50 --warmup 10 --cpu-baseline off > gpurun_out/abc/c${c}_z${z}_$rep.log 2>&1 || exit 1
      tail -1 gpurun_out/abc/c${c}_z${z}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg$c z=$z', d['value'], d['ms_per_step'], d['fwd_bwd_ms_per_view'])"
    done
  done
done
