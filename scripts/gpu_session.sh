set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ -p no:cacheprovider > gpurun_out/t7.log 2>&1; rc=$?; tail -3 gpurun_out/t7.log; [ $rc -ne 0 ] && exit $rc
BENCH_ARGS="--steps 100 --warmup 10" bash scripts/ab_bench.sh > gpurun_out/ab7.log 2>&1; rc=$?; grep -E "==|views" gpurun_out/ab7.log; grep -A1 "==" gpurun_out/ab7.log | grep -v views | head -0
GSD_DP_ONE_RANK=1 timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-baseline off > gpurun_out/dp7.log 2>&1; rc=$?; grep metric gpurun_out/dp7.log | cut -c1-250; exit $rc
