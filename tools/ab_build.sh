#!/bin/bash
# A/B builds of libmbrwt.so (measurement only, never shipped as the product):
#   tools/ab_build.sh NAME "-DMBRWT_AB_X -DMBRWT_AB_Y" [source.hip ...]
# recompiles the named sources (default csrc/rows.hip) with the extra defines
# and links them with the release objects of genome_graph_annotation_amd/_build
# into tools/_ab/libmbrwt_NAME.so (load it with MBRWT_LIB=...).
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
NAME="$1"; DEFS="$2"; shift 2
SRCS=("$@"); [ ${#SRCS[@]} -eq 0 ] && SRCS=(csrc/rows.hip)
PKG="$ROOT/genome_graph_annotation_amd"
make -s -C "$PKG" >/dev/null
OUT="/tmp/mbrwt_ab_obj_$NAME"; mkdir -p "$OUT" "$ROOT/tools/_ab"
HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-result"
objs=()
for o in "$PKG"/_build/*.o; do
  b="$(basename "$o" .o)"; skip=0
  for s in "${SRCS[@]}"; do [ "$(basename "$s")" = "$b" ] && skip=1; done
  [ $skip -eq 0 ] && objs+=("$o")
done
for s in "${SRCS[@]}"; do
  /opt/rocm/bin/hipcc $HIPFLAGS $DEFS -x hip -c "$PKG/$s" -o "$OUT/$(basename "$s").o"
  objs+=("$OUT/$(basename "$s").o")
done
/opt/rocm/bin/hipcc $HIPFLAGS -shared -o "$ROOT/tools/_ab/libmbrwt_$NAME.so" "${objs[@]}"
echo "tools/_ab/libmbrwt_$NAME.so"
