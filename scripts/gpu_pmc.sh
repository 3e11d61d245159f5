#!/bin/bash
# PMC counter passes (each its own rocprofv3 run; no tracing domains besides kernel trace).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; O="${PMC_OUT:-gpurun_out/pmc}"; mkdir -p "$O"
export TMPDIR=/tmp
if [ -n "$LIST" ]; then rocprofv3 -L > "$O/counters.txt" 2>&1; fi
i=0
IFS=';' read -ra PASSES <<< "${PMC_PASSES}"
for pass in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-include-regex "${KREGEX:-gsd}" --output-format csv \
      -d "$R/$O/p$i" -o pmc -- python "$R/${PROF_SCRIPT:-scripts/prof_render.py}" ${PROF_ARGS:---iters 3} > "$O/p$i.log" 2>&1
  rc=$?; echo "pass $i ($pass) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$O/p$i.log"; exit $rc; }
done
exit 0
