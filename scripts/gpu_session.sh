set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_multiview.py tests/test_gpu_parity.py -k "views or rank or ranks" -p no:cacheprovider > gpurun_out/t9.log 2>&1; rc=$?; tail -3 gpurun_out/t9.log; [ $rc -ne 0 ] && exit $rc
export GSD_DP_ONE_RANK=1
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-baseline off > gpurun_out/dp9.log 2>&1; rc=$?; grep metric gpurun_out/dp9.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['kernels_ms'])"; exit $rc
