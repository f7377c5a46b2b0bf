#!/bin/bash
# Build tools/run/w43_bench (+ variants) here on the CPU (OUT=dir to override;
# tools/run travels to the GPU box, tools/bin does not — empty tools/run after use): the F(2,3) / direct
# conv objects once, conv_wino43.hip per variant.
#   tools/build_w43.sh                 -> tools/run/w43_bench
#   VARIANTS="abl1:-DSEDX_W43_ABL=1 abl2:-DSEDX_W43_ABL=2" tools/build_w43.sh
set -e
cd "$(dirname "$0")/.."
C=sound-event-detection_amd/csrc
O=${OUT:-tools/run}
mkdir -p $O
H="/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value -fno-slp-vectorize -fno-vectorize -I$C"
for src in conv conv_wino; do
  if [ ! -f $O/$src.o ] || [ $C/$src.hip -nt $O/$src.o ] || [ $C/sedx_internal.h -nt $O/$src.o ]; then
    $H -c $C/$src.hip -o $O/$src.o &
  fi
done
[ tools/wino43_bench.cpp -nt $O/wino43_bench.o ] || [ ! -f $O/wino43_bench.o ] && $H -c tools/wino43_bench.cpp -o $O/wino43_bench.o &
build_variant() {   # name flags (a SEDX_W43_STAMPS variant gets its own bench object, which prints the stamps)
  local bo=$O/wino43_bench.o
  if [[ "$2" == *SEDX_W43_STAMPS* ]]; then bo=$O/wino43_bench_$1.o; $H $2 -c tools/wino43_bench.cpp -o $bo || return 1; fi
  $H $2 -c $C/conv_wino43.hip -o $O/w43_$1.o && $H -o $O/w43_bench${1:+_$1} $bo $O/conv.o $O/conv_wino.o $O/w43_$1.o
}
wait
pids=()
[ -n "$NO_DEFAULT" ] || { build_variant "" "" & pids+=($!); }
for vf in $VARIANTS; do n=${vf%%:*}; f=${vf#*:}; build_variant "$n" "${f//,/ }" & pids+=($!); done
for p in "${pids[@]}"; do wait $p; done
ls -la $O
