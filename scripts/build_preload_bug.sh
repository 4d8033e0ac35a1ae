#!/bin/bash
# Builds build/bug/preload_bug.so: the library of this tree with ONLY the
# 4-wave index-preload fix of fd7563c undone (num_records = the exact byte
# size of the index list, so with an odd entry count the last entry reads 0;
# the ADVICE r04 range guard in kblock_of removed too). It reproduces the bug
# the f327921 library shipped with, on today's sources, so that the parity
# tests (tests/test_gpu_fuzz.py, test_gpu_configs.py) can be shown to catch
# it: SPUTNIK_AMD_LIB=build/bug/preload_bug.so python -m pytest ...
set -e
ROOT=$(cd $(dirname $0)/.. && pwd)
D=$ROOT/build/bug/preload_bug
rm -rf $D && mkdir -p $D/csrc
cp $ROOT/sputnik_amd/csrc/*.hip $ROOT/sputnik_amd/csrc/*.cpp $ROOT/sputnik_amd/csrc/*.h $ROOT/sputnik_amd/csrc/*.inc $D/csrc/
sed -i 's/(nb_all \* 2 + 3) & ~3/nb_all * 2/' $D/csrc/dsd4w.hip
sed -i 's/if (!idx_pre || e >= nb_all) return/if (!idx_pre) return/' $D/csrc/dsd4w.hip
grep -q 'make_buffer_rsrc(' $D/csrc/dsd4w.hip
if grep -q 'nb_all \* 2 + 3' $D/csrc/dsd4w.hip || grep -q 'e >= nb_all' $D/csrc/dsd4w.hip; then
  echo "patch did not apply" >&2; exit 1
fi
grep -n 'nb_all \* 2, 0x' $D/csrc/dsd4w.hip
for f in block_gemm dsd4w metadata dispatch c_api; do
  src=$D/csrc/$f.hip; [ -f $src ] || src=$D/csrc/$f.cpp
  /opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -I$ROOT/include \
    -DSPUTNIK_BUILD_HASH=\"preload_bug\" -x hip -c $src -o $D/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/build/bug/preload_bug.so $D/*.o
echo built $ROOT/build/bug/preload_bug.so
