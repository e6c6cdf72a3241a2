#!/bin/bash
# usage (here, CPU): tools/build_variant.sh <name> <src.hip> [hipcc flags...]
# -> build_ab/libpemp_<name>.so: csrc/*.o with <src>'s object rebuilt under the extra flags
# (A/B on the GPU box: PEMP_LIB=build_ab/libpemp_<name>.so, e.g. through tools/ab_env.sh / tools/mpn_ab.py).
# <src.hip> is a csrc file name (mpn.hip) or a path to another copy of it; REPLACE=<object stem> names the csrc
# object it stands in for when the stem differs (REPLACE=mpn for /tmp/mpn_base.hip).
set -e
name=$1; src=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
csrc=$root/pose-estimation-with-message-passing-networks_amd/csrc
mkdir -p "$root/build_ab"
base=${REPLACE:-$(basename "$src" .hip)}
if [ -f "$src" ]; then path=$(cd "$(dirname "$src")" && pwd)/$(basename "$src"); else path=$csrc/$base.hip; fi
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DOCML_BASIC_ROUNDED_OPERATIONS -Wno-unused-function -Wno-unused-variable \
  -I"$root/include" -I"$csrc" "$@" -c "$path" -o "$root/build_ab/v_${name}_$base.o"
objs=""
for o in "$csrc"/*.o; do
  [ "$(basename "$o")" = "$base.o" ] || objs="$objs $o"
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$root/build_ab/libpemp_$name.so" $objs \
  "$root/build_ab/v_${name}_$base.o"
echo "build_ab/libpemp_$name.so"
