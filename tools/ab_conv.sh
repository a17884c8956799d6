# GPU: conv tests on the default build, then tools/conv_bench.py against builds
# lightzero_amd/liblzm_var<X>.so (LZM_LIB), interleaved. usage: bash tools/ab_conv.sh OUT KIND REPS A B ...
set -e
out=$1; kind=$2; reps=$3; shift 3
mkdir -p "$out"
for rep in $(seq $reps); do for v in "$@"; do
  LZM_LIB=lightzero_amd/liblzm_var$v.so timeout -k 10 200 python tools/conv_bench.py --kind $kind --searches 20 > "$out/${kind}_${v}_$rep.json" 2>&1
  python3 -c "import json;d=json.loads(open('$out/${kind}_${v}_$rep.json').read().strip().splitlines()[-1]);print('$kind $v $rep', d['value'])" | tee -a "$out/summary.txt"
done; done
