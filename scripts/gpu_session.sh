set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/dp; export TMPDIR=/tmp
GSD_DIST_BACKEND=gloo HSA_ENABLE_IPC_MODE_LEGACY=0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/dp/b2.log 2>&1 || { tail -20 gpurun_out/dp/b2.log; exit 1; }
grep '"metric"' gpurun_out/dp/b2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('exchange'))"
GSD_DP_ONE_RANK=1 HSA_ENABLE_IPC_MODE_LEGACY=0 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/dp/b1.log 2>&1 || { tail -20 gpurun_out/dp/b1.log; exit 1; }
grep '"metric"' gpurun_out/dp/b1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d.get('exchange'))"
