#!/bin/bash
# Experiment: build libgsd_hip.so variants with -D flags into /tmp and time the kernels
# with scripts/prof_render.py (timing via gsd_timing).  VARIANTS="name:-DFLAG ..." separated by ';'.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
IFS=';' read -ra VS <<< "${VARIANTS}"
for v in "base:" "${VS[@]}"; do
  name="${v%%:*}"; flags="${v#*:}"
  out="/tmp/gsdvar_$name"; mkdir -p "$out"
  make -s -C gaussian-splatting_deformable_amd/csrc OUT="$out" HIPFLAGS_EXTRA="$flags" -j16 > "$out/build.log" 2>&1 || { echo "build $name failed"; tail "$out/build.log"; exit 1; }
  GSD_SKIP_BUILD_ID=1 GSD_HIP_LIB="$out/libgsd_hip.so" timeout -k 10 300 ${PROF_CMD:-python scripts/prof_render.py --iters ${ITERS:-20} --timing} > gpurun_out/exp_$name.log 2>&1
  rc=$?; echo "== $name ($flags) rc=$rc"; tail -12 gpurun_out/exp_$name.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
