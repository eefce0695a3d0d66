# Build variant libraries of libmcs_amd.so with extra -D flags for extractor tuning runs
# (tools/gpu/variants.sh).  Usage: tools/build_variants.sh NAME "FLAGS" [NAME "FLAGS" ...]
# Each variant recompiles the extractor sources with FLAGS into lib/var_NAME/libmcs_amd.so.
set -e
cd "$(dirname "$0")/.."
P=multicol-slam-annotation_amd
EXTR=${EXTR:-"extractor.hip k_pyramid.hip k_fast_rows.hip k_octree.hip k_desc.hip extractor_plan.cpp hamming.hip"}
while [ $# -ge 2 ]; do
  NAME=$1; FLAGS=$2; shift 2
  D=$P/lib/var_$NAME; rm -rf $D; mkdir -p $D
  for f in $P/lib/*.o; do cp $f $D/; done
  for s in $EXTR; do
    LANG=""; case $s in *.hip) LANG="-x hip";; esac
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-function $FLAGS -I include -c $LANG $P/csrc/$s -o $D/$s.o
  done
  hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libmcs_amd.so $D/*.o
  echo "built $D ($FLAGS)"
done
