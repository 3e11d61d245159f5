#!/bin/bash
# A/B of prebuilt library variants (built on the CPU side into gaussian-splatting_deformable_amd/build_*/, shipped
# with the tree): LIBS="name:dir name:dir ..." timed with scripts/prof_render.py --timing (REPS rounds, alternating),
# or with PROF_CMD.  Variants are other sources or flags than the tree's, so GSD_SKIP_BUILD_ID=1.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-ab}"; mkdir -p "$O"
for rep in $(seq 1 ${REPS:-3}); do
  for v in $LIBS; do
    name="${v%%:*}"; dir="${v#*:}"
    GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB="$dir/libgsd_hip.so" timeout -k 10 300 \
        ${PROF_CMD:-python scripts/prof_render.py --iters ${ITERS:-30} --timing ${PROF_ARGS}} > "$O/${name}_$rep.log" 2>&1 \
        || { echo "== $name rep $rep failed"; tail -20 "$O/${name}_$rep.log"; exit 1; }
    echo "== $name rep $rep: $(grep -E '^render_(fwd|bwd)' "$O/${name}_$rep.log" | awk '{printf "%s %s  ", $1, $2}')"
  done
done
exit 0
