# GPU: DownSample per-layer kernel times (tools/repr_bench.py, B = 256, rocprofv3 --kernel-trace --stats) for
# library builds: "cur" = lightzero_amd/liblzmcts.so, X = lightzero_amd/liblzm_varX.so (LZM_LIB), interleaved
# twice. usage: bash tools/repr_ab.sh OUT TAG...
set -e
out=$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for v in "$@"; do
    lib=lightzero_amd/liblzmcts.so
    [ "$v" != cur ] && lib=lightzero_amd/liblzm_var$v.so
    LZM_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$out/${v}_$rep" -o t --output-format csv -- \
      python3 tools/repr_bench.py --batches 256 --reps 20 > "$out/${v}_$rep.log" 2>&1
    echo "$v $rep $(grep us_per_downsample $out/${v}_$rep.log)" >> "$out/summary.txt"
  done
done
cat "$out/summary.txt"
