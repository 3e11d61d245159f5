set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ -p no:cacheprovider > gpurun_out/t20.log 2>&1; rc=$?; tail -2 gpurun_out/t20.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/bench_v30.log 2>&1; rc=$?; tail -1 gpurun_out/bench_v30.log | cut -c1-200; exit $rc
