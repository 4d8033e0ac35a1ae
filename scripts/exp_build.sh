#!/bin/bash
# Build ablation/variant libraries: scripts/exp_build.sh name:FLAGS ...
# e.g. base:-DSPUTNIK_EXP=0 nomfma:-DSPUTNIK_EXP=1. Output build/exp/<name>.so
set -e
ROOT=$(cd $(dirname $0)/.. && pwd)
mkdir -p $ROOT/build/exp
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  d=$ROOT/build/exp/$name; mkdir -p $d
  for f in block_gemm dsd4w metadata dispatch c_api; do
    src=$ROOT/sputnik_amd/csrc/$f.hip; [ -f $src ] || src=$ROOT/sputnik_amd/csrc/$f.cpp
    /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -I$ROOT/include $flags -x hip -c $src -o $d/$f.o &
    pids="$pids $!"
  done
  for p in $pids; do wait $p || { echo "build of $name failed"; exit 1; }; done
  pids=""
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/build/exp/$name.so $d/*.o
  echo built $name
done
