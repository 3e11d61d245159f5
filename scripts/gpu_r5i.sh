#!/bin/bash
# Round 5: the tightened parity bar (flip statistics into parity_flips.jsonl), the MLP tests (evaluation kernel,
# fallback kernels), and the evaluation timings at 1M Gaussians next to torch f32.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r5i}"; mkdir -p "$O"
export GSD_PARITY_REPORT="$O/parity_flips.jsonl"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_render_modes.py \
    tests/test_gpu_mlp.py -x -q -p no:cacheprovider --timeout 600 --timeout-method thread > "$O/tests.log" 2>&1 \
    || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
for v in "" ; do :; done
timeout -k 10 200 python scripts/time_mlp_fwd.py --eval > "$O/mlp_eval.txt" 2>&1 || { tail -5 "$O/mlp_eval.txt"; exit 1; }
GSD_MLP_TORCH=1 timeout -k 10 200 python scripts/time_mlp_fwd.py --eval >> "$O/mlp_eval.txt" 2>&1 || { tail -5 "$O/mlp_eval.txt"; exit 1; }
timeout -k 10 200 python scripts/time_mlp_fwd.py >> "$O/mlp_eval.txt" 2>&1 || { tail -5 "$O/mlp_eval.txt"; exit 1; }
grep -v amdgpu.ids "$O/mlp_eval.txt"
echo done
