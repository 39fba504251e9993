# Build the working tree's library with extra compiler flags into lib_$1/
# for a process-level A/B (tools/ab_libs.sh LIBS="$1 ..."):
#   bash tools/build_variant.sh nd -DHPCCG_NO_WAITER_DRAIN
set -e
NAME=$1; shift
D=$(mktemp -d /tmp/hpccg_var.XXXX)
cp -r hpccg-sycl_amd include "$D/"
rm -rf "$D/hpccg-sycl_amd/build" "$D/hpccg-sycl_amd/lib" "$D/hpccg-sycl_amd/bin"
make -C "$D/hpccg-sycl_amd" -j8 CXXFLAGS_EXTRA="$*" HIPFLAGS_EXTRA="$*" >/dev/null
mkdir -p "lib_$NAME"
cp "$D/hpccg-sycl_amd/lib/libhpccg_hip.so" "lib_$NAME/"
rm -rf "$D"
echo "lib_$NAME/libhpccg_hip.so: $*"
