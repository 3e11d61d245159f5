set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/final7; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final7/gpu_tests.log 2>&1; rc=$?
tail -2 gpurun_out/final7/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --config 5 --steps 300 --warmup 5 --cpu-baseline off > gpurun_out/final7/b5.log 2>&1 || exit 1
tail -1 gpurun_out/final7/b5.log | cut -c1-200
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final7/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/final7/smoke.log
