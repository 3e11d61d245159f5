set -o pipefail
mkdir -p gpurun_out/ab
for rep in 1 2 3; do
  for z in 1 0; do
    GSD_FWD_ZERO_SCRATCH=$z timeout -k 10 300 python3 bench.py --steps ${STEPS:-20} --warmup 5 --cpu-baseline off > gpurun_out/ab/z${z}_$rep.log 2>&1 || exit 1
    tail -1 gpurun_out/ab/z${z}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('z=$z', d['value'], d['ms_per_step'], d['fwd_bwd_ms_per_view'])"
  done
done
