#!/bin/bash
# PMC counter passes (each its own rocprofv3 run; no tracing domains besides kernel trace).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
if [ -n "$LIST" ]; then rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1; fi
i=0
IFS=';' read -ra PASSES <<< "${PMC_PASSES}"
for pass in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-include-regex "${KREGEX:-gsd}" --output-format csv \
      -d "$R/gpurun_out/pmc/p$i" -o pmc -- python "$R/${PROF_SCRIPT:-scripts/prof_render.py}" ${PROF_ARGS:---iters 3} > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($pass) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/pmc/p$i.log; exit $rc; }
done
exit 0
