set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/cs; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py > gpurun_out/cs/t.log 2>&1; rc=$?; tail -1 gpurun_out/cs/t.log; [ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/cs/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cs/prof -o b -- python3 bench.py --steps 30 --warmup 5 --cpu-baseline off > gpurun_out/cs/b.log 2>&1 || exit 1
grep -o '"gsd::k_tile_scan[^,]*,[0-9]*,[0-9]*,[0-9.]*' gpurun_out/cs/prof/b_kernel_stats.csv
