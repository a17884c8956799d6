# GPU: Breakout collect-step bench and Pong EZ search bench for several library builds ("cur" =
# liblzmcts.so, X = liblzm_varX.so), interleaved twice. usage: bash tools/gpu_ab_conv_libs.sh OUT TAG...
set -e
out=$1; shift
mkdir -p $out
for rep in 1 2; do
  for v in "$@"; do
    lib=lightzero_amd/liblzmcts.so
    [ "$v" != cur ] && lib=lightzero_amd/liblzm_var$v.so
    LZM_LIB=$lib timeout -k 10 200 python bench.py --workload breakout --step collect --steps 20 --warmup 3 --no-cpu-baseline --configs none > $out/b5_${v}_$rep.json 2>&1
    LZM_LIB=$lib timeout -k 10 200 python tools/conv_bench.py --kind ez --searches 10 > $out/c3_${v}_$rep.json 2>&1
    python3 -c "import json;d=json.loads(open('$out/b5_${v}_$rep.json').read().strip().splitlines()[-1]);e=json.loads(open('$out/c3_${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', $rep, 'config5', d['value'], d['ms_per_step'], 'ez', e['value'], e.get('ms_per_search'))" >> $out/summary.txt
  done
done
cat $out/summary.txt
