# Build the library of git revision $1 (default HEAD) into lib_base/ for an
# A/B against the working tree (HPCCG_HIP_LIB=lib_base/libhpccg_hip.so).
set -e
REV=${1:-HEAD}
D=$(mktemp -d /tmp/hpccg_base.XXXX)
git archive "$REV" | tar -x -C "$D"
make -C "$D/hpccg-sycl_amd" -j8 >/dev/null
mkdir -p lib_base
cp "$D/hpccg-sycl_amd/lib/libhpccg_hip.so" lib_base/
rm -rf "$D"
echo "lib_base/libhpccg_hip.so from $REV"
