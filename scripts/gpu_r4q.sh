#!/bin/bash
# Round 4: scatter with nontemporal reads (build_nt, -DGSD_SCATTER_NT=1) against the product -- parity tests with
# it, kernel times (A/B/A over scripts/prof_render.py) and WRITE_SIZE / FETCH_SIZE passes on k_scatter_hist.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r4q}"; mkdir -p "$O"
NT=$PWD/gaussian-splatting_deformable_amd/build_nt/libgsd_hip.so
BASE=$PWD/gaussian-splatting_deformable_amd/build/libgsd_hip.so
GSD_HIP_LIB=$NT timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
i=0
for lib in $BASE $NT $BASE; do
  i=$((i+1))
  GSD_HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/p$i" -o run -- \
      python3 scripts/prof_render.py --iters 30 > "$O/t$i.log" 2>&1 || { tail -20 "$O/t$i.log"; exit 1; }
  find "$O/p$i" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$O/stats_$i.csv"
  python3 scripts/kstats.py --match scatter_hist "$O/stats_$i.csv"
done
j=0
for lib in $BASE $NT; do
  for c in WRITE_SIZE FETCH_SIZE; do
    j=$((j+1))
    GSD_HIP_LIB=$lib timeout -s KILL 90 rocprofv3 --pmc $c --kernel-include-regex scatter_hist --output-format csv \
        -d "$O/m$j" -o pmc -- python3 scripts/prof_render.py --iters 3 > "$O/m$j.log" 2>&1 || { tail -5 "$O/m$j.log"; exit 1; }
    f=$(find "$O/m$j" -name '*counter_collection.csv' | head -1)
    python3 -c "
import csv,sys
rows=[r for r in csv.DictReader(open('$f'))]
v=[float(r['Counter_Value']) for r in rows if r['Counter_Name']=='$c']
n=len(set(r['Dispatch_Id'] for r in rows))
print('$lib'.split('/')[-2], '$c', round(sum(v)/max(n,1)), 'KB per dispatch', n)"
  done
done
