#!/bin/bash
# Round 4: MLP head outputs + in-place gradients -- the MLP / training GPU tests, the MLP-live bench line and its
# kernel statistics.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-r4j}"; mkdir -p "$O"
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_mlp.py \
    tests/test_gpu_train.py > "$O/tests.log" 2>&1 || { tail -40 "$O/tests.log"; exit 1; }
tail -3 "$O/tests.log"
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --with-mlp --cpu-baseline off > "$O/bench_mlp.log" 2>&1 \
    || { tail -20 "$O/bench_mlp.log"; exit 1; }
tail -1 "$O/bench_mlp.log" | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --gpus 1 \
    --steps 10 --warmup 3 --with-mlp --cpu-baseline off > "$O/bench_prof.log" 2>&1 || { tail -20 "$O/bench_prof.log"; exit 1; }
find "$O/prof" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$O/kernel_stats.csv"
