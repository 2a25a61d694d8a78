# Build a variant of libsphhip.so for an interleaved A/B: bash scripts/build_variant.sh NAME "-DKNOB=..."
# -> build/variants/lib_NAME.so (objects in build/obj_NAME, removed afterwards). "head" = no flags.
set -e
cd "$(dirname "$0")/.."
name=$1; extra=${2:-}
mkdir -p build/variants
make -s -j8 -C sph-test_amd/csrc OBJDIR=../../build/obj_$name OUT=../../build/variants/lib_$name.so EXTRA="$extra"
rm -rf build/obj_$name
echo "built build/variants/lib_$name.so ($extra)"
