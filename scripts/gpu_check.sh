#!/bin/bash
# GPU-box check: smoke() then the -m gpu parity tests.  Stops at the first
# step that dies abnormally (fault / abort / timeout): only rc 0 or 1 continue.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/smoke.log
if [ $rc -gt 1 ]; then echo "smoke died rc=$rc"; exit $rc; fi
timeout -k 10 1000 python -m pytest tests -q -m gpu -p no:cacheprovider ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc2=$?; echo "tests rc=$rc2" >> gpurun_out/gpu_tests.log
tail -5 gpurun_out/smoke.log; tail -30 gpurun_out/gpu_tests.log
exit $(( rc > rc2 ? rc : rc2 ))
