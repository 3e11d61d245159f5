#!/bin/bash
# GPU-box bench: parity subset, bench.py (N=1), then a rocprofv3 kernel-trace of a short bench.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
if [ -n "${TESTS}" ]; then
  timeout -k 10 600 python -m pytest ${TESTS} -q -m gpu -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc" >> gpurun_out/gpu_tests.log; tail -3 gpurun_out/gpu_tests.log
  [ $rc -gt 1 ] && exit $rc
fi
timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
if [ -n "${PROF}" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o bench -- \
      python "$R/bench.py" --steps 10 --warmup 3 --cpu-baseline off > gpurun_out/prof.log 2>&1
  rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof.log
  find gpurun_out/prof -name "*stats*" | head
fi
exit $rc
