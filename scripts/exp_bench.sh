#!/bin/bash
# Experiment: bench.py with libgsd_hip.so variants built with -D flags (VARIANTS="name:-DFLAG;...").
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
IFS=';' read -ra VS <<< "${VARIANTS}"
for v in "base:" "${VS[@]}"; do
  name="${v%%:*}"; flags="${v#*:}"
  out="/tmp/gsdvar_$name"; mkdir -p "$out"
  make -s -C gaussian-splatting_deformable_amd/csrc OUT="$out" HIPFLAGS_EXTRA="$flags" -j16 > "$out/build.log" 2>&1 || { echo "build $name failed"; tail "$out/build.log"; exit 1; }
  GSD_HIP_LIB="$out/libgsd_hip.so" timeout -k 10 600 python bench.py --cpu-baseline off ${BENCH_ARGS} > gpurun_out/expbench_$name.log 2>&1
  rc=$?; echo "== $name ($flags) rc=$rc"; tail -1 gpurun_out/expbench_$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('views/s', d['value'], 'ms/step', d['ms_per_step'], 'fwd_bwd', d['fwd_bwd_ms_per_view'])"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
