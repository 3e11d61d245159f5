#!/bin/bash
# Round 4: MLP kernel iteration -- the MLP GPU tests, then the kernel statistics of scripts/mlp_ablate.py (P = 1M).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r4l}"; mkdir -p "$O"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mlp.py \
    > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/p" -o run -- \
    python3 scripts/mlp_ablate.py --reps 5 > "$O/abl.log" 2>&1 || { tail -20 "$O/abl.log"; exit 1; }
find "$O/p" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$O/stats.csv"
grep "ms per" "$O/abl.log"
python3 - "$O/stats.csv" <<'PY'
import csv, sys
for r in sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r['TotalDurationNs'])):
    if 'mlp' in r['Name']: print('%9.1f us x %4s  %s' % (float(r['AverageNs']) / 1e3, r['Calls'], r['Name'][:70]))
PY
