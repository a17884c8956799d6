# Build lightzero_amd/liblzm_var<NAME>.so from the sources of git revision REV (default: the working tree),
# for interleaved A/B runs (tools/ab_libs.sh). usage: bash tools/build_variant.sh NAME [REV] [extra hipcc flags]
set -e
name=$1; rev=${2:-}; shift; shift || true
root=$(cd "$(dirname "$0")/.." && pwd)
src=$root
if [ -n "$rev" ]; then
  src=$(mktemp -d /tmp/lzm_var_XXXX)
  git -C "$root" archive "$rev" lightzero_amd/csrc include | tar -x -C "$src"
fi
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -shared -Wall --offload-arch=gfx950 "$@" \
  -o "$root/lightzero_amd/liblzm_var$name.so" "$src/lightzero_amd/csrc/lzm_kernels.hip"
echo "built lightzero_amd/liblzm_var$name.so from ${rev:-working tree}"
