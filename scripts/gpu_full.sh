#!/bin/bash
# Full GPU-box pass at HEAD: the -m gpu tests, smoke(), the driver's bench command and a rocprofv3
# kernel-trace summary of it.  OUT names the directory under gpurun_out/.  Each GPU step has its
# own time limit and the chain stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; export TMPDIR=/tmp
O="gpurun_out/${OUT:-full}"; mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    ${PYTEST_ARGS} > "$O/gpu_tests.log" 2>&1 || { tail -30 "$O/gpu_tests.log"; exit 1; }
tail -3 "$O/gpu_tests.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver.log" 2>&1 || { tail -20 "$O/bench_driver.log"; exit 1; }
tail -1 "$O/bench_driver.log" | cut -c1-400
if [ -n "$PROF" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off \
      > "$O/bench_prof.log" 2>&1 || { tail -20 "$O/bench_prof.log"; exit 1; }
  find "$O/prof" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$O/kernel_stats.csv"
fi
echo done
