set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for c in 3 1 2 5; do
  timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 5 --cpu-baseline off > gpurun_out/bench_cfg$c.log 2>&1; rc=$?
  echo "cfg $c rc=$rc"; grep metric gpurun_out/bench_cfg$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['fwd_bwd_ms_per_view'], d['config']['workload'][:90], d['config']['num_rendered'])"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_cfg$c.log; exit $rc; }
done
exit 0
