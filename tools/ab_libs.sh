# GPU: bench.py against several builds of the library (lightzero_amd/liblzm_var<X>.so, LZM_LIB),
# twice each, interleaved. usage: bash tools/ab_libs.sh OUT_DIR A B:ENV=VAL C ...
# (a variant X:ENV=VAL runs build X with that environment variable set; AB_ARGS: extra bench.py args)
set -e
out=$1; shift
mkdir -p "$out"
for rep in 1 2; do
  for v in "$@"; do
    lib=${v%%:*}
    envs=""
    if [[ "$v" == *:* ]]; then envs=${v#*:}; fi
    tag=$(echo "$v" | tr ':=' '__')
    env $envs LZM_LIB=lightzero_amd/liblzm_var$lib.so timeout -k 10 200 python bench.py --no-cpu-baseline --secondary none --configs none --steps 30 $AB_ARGS > "$out/b_${tag}_$rep.json" 2>&1
    python3 -c "import json,sys;d=json.loads(open('$out/b_${tag}_$rep.json').read().strip().splitlines()[-1]);print('$v', $rep, d['value'], d['roofline']['launch_us'], d['tie_stream_errors'])" >> "$out/summary.txt"
  done
done
cat "$out/summary.txt"
