set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 0 1 0 1; do
if [ $v = 1 ]; then export GSD_BENCH_BARE_BACKWARD=1; else unset GSD_BENCH_BARE_BACKWARD; fi
timeout -k 10 200 python bench.py --steps 300 --warmup 20 --cpu-baseline off > gpurun_out/b_$v.log 2>&1 || exit 1
python - "$v" <<'PY'
import json,sys
d=json.loads(open(f"gpurun_out/b_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print("bare" if sys.argv[1]=="1" else "seed", d["value"], d["ms_per_step"], d["fwd_bwd_ms_per_view"], d["kernels_ms"]["l1_ssim"])
PY
done
