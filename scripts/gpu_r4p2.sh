#!/bin/bash
# Round 4: matrix-core busy fraction of the network's fused kernels -- one PMC pass (SQ_VALU_MFMA_BUSY_CYCLES,
# GRBM_GUI_ACTIVE) over scripts/mlp_ablate.py (P = 1M, 2 reps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r4p2}"; mkdir -p "$O"
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "k_mlp_(fwd_fused|bwd_chain|wgrad<)" \
    --output-format csv -d "$O/m" -o pmc -- python3 scripts/mlp_ablate.py --reps 2 > "$O/pmc.log" 2>&1 || { tail -10 "$O/pmc.log"; exit 1; }
f=$(find "$O/m" -name '*counter_collection.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
for r in rows:
    k = r['Kernel_Name'].split('(')[0]
    agg[k][r['Counter_Name']] += float(r['Counter_Value']); n[k].add(r['Dispatch_Id'])
for k, c in agg.items():
    d = len(n[k]); busy = c['SQ_VALU_MFMA_BUSY_CYCLES'] / d; gui = c['GRBM_GUI_ACTIVE'] / d
    # MFMA busy cycles summed over the 1024 SIMDs; GRBM_GUI_ACTIVE summed over the 8 XCDs
    print('%-45s dispatches %d  mfma_busy_frac %.3f' % (k[-45:], d, busy / (1024.0 * gui / 8.0)))
PY
