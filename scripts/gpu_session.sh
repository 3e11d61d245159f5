set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/w2; export TMPDIR=/tmp
for g in 0 1 0 1 0 1; do
GSD_BENCH_PRIME=$g GSD_BENCH_STEP_TIMES=1 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/w2/b.log 2> gpurun_out/w2/s.log || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/w2/b.log').read().strip().splitlines()[-1]); print('prime $g', d['value'], d['ms_per_step'])"
grep "step ms" gpurun_out/w2/s.log | cut -c1-60
done
