set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_configs.py -p no:cacheprovider > gpurun_out/t17.log 2>&1; rc=$?; tail -2 gpurun_out/t17.log; [ $rc -ne 0 ] && exit $rc
RENDER=1 ITERS=30 bash scripts/ab_bench.sh > gpurun_out/ab17r.log 2>&1 || exit 1
grep -E "==|render_|preprocess_fwd" gpurun_out/ab17r.log
