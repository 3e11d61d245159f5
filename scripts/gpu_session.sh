set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_train.py tests/test_gpu_parity.py -p no:cacheprovider > gpurun_out/t6.log 2>&1; rc=$?; tail -3 gpurun_out/t6.log; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--steps 100 --warmup 10" bash scripts/ab_bench.sh > gpurun_out/ab6.log 2>&1; rc=$?; grep -E "==|views" gpurun_out/ab6.log; exit $rc
