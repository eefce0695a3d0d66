# Build ablated variants of libmcs_amd.so (k_pyr_fast with -DMCS_ABLATE=N) for tools/gpu/ablate.sh.
set -e
cd "$(dirname "$0")/.."
P=multicol-slam-annotation_amd
for N in 1 2; do
  D=$P/lib/abl$N; mkdir -p $D
  for f in $P/lib/*.o; do cp $f $D/; done
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DMCS_ABLATE=$N -I include -c -x hip $P/csrc/k_pyramid.hip -o $D/k_pyramid.hip.o
  hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libmcs_amd.so $D/*.o
done
