#!/bin/bash
# Build a variant of libpfm_hip.so with one source recompiled under extra defines, for A/B runs (PFM_LIB):
#   tools/build_variant.sh NAME SRC.hip -DMACRO=V ...   -> abvar/NAME/libpfm_hip.so (git-ignored, outside the product
#   package; delete after the A/B)
set -e
name=$1; src=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
python -c "import sys; sys.path.insert(0, '$R'); import funasr_amd.build as b; b.build()" > /dev/null
out=$R/abvar/$name; mkdir -p $out
objs=""
for o in $R/funasr_amd/_lib/obj/*.o; do
  if [ "$(basename $o)" = "$(basename $src).o" ]; then
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Wno-unused-variable \
      -Wno-unused-lambda-capture -I $R/include "$@" -c $R/funasr_amd/csrc/$src -o $out/$(basename $o)
    objs="$objs $out/$(basename $o)"
  else
    objs="$objs $o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libpfm_hip.so $objs
echo $out/libpfm_hip.so
