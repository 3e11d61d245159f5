#!/bin/bash
# Round 4: cProfile of bench.py --config 1 (host-bound) with the round-3 tree and HEAD: where the extra host time goes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="$PWD/gpurun_out/${OUT:-r4m3}"; mkdir -p "$O"
for t in .ab/r3 .; do
  n=$(basename $(realpath $t))
  (cd $t && timeout -k 10 300 python3 -m cProfile -o "$O/prof_$n.out" bench.py --config 1 --steps 50 --warmup 10 \
      --cpu-baseline off) > "$O/b_$n.log" 2>&1 || { tail -20 "$O/b_$n.log"; exit 1; }
  python3 -c "
import pstats; s=pstats.Stats('$O/prof_$n.out'); s.sort_stats('tottime').print_stats(25)" > "$O/top_$n.txt" 2>&1
  tail -1 "$O/b_$n.log" | cut -c1-120
done
