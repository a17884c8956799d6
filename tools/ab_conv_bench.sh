# GPU: tools/conv_bench.py against two library builds (lightzero_amd/liblzm_var<X>.so, LZM_LIB), interleaved
# twice each. usage: bash tools/ab_conv_bench.sh OUT_DIR KIND A B ...
set -e
out=$1; kind=$2; shift 2
mkdir -p "$out"
for rep in 1 2; do
  for v in "$@"; do
    LZM_LIB=lightzero_amd/liblzm_var$v.so timeout -k 10 200 python tools/conv_bench.py --kind $kind --searches 20 \
      > "$out/c_${v}_$rep.json" 2>&1
    python3 -c "import json;d=json.loads(open('$out/c_${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', $rep, d['value'], d.get('ms_per_search'))" >> "$out/summary.txt"
  done
done
cat "$out/summary.txt"
