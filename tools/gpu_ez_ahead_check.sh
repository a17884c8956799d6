# GPU: the conv / config 3 / divergence GPU tests on this build (the EZ search at read-ahead 5), then the Pong
# EZ search bench against lightzero_amd/liblzm_varB.so (read-ahead 3), interleaved twice, then the default
# bench line. usage: bash tools/gpu_ez_ahead_check.sh OUT
set -e
out=$1
mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_config3.py tests/test_gpu_divergence.py > $out/t.log 2>&1
for rep in 1 2; do
  for v in cur B; do
    lib=lightzero_amd/liblzmcts.so
    [ "$v" != cur ] && lib=lightzero_amd/liblzm_var$v.so
    LZM_LIB=$lib timeout -k 10 200 python tools/conv_bench.py --kind ez --searches 10 > $out/c3_${v}_$rep.json 2>&1
    python3 -c "import json;e=json.loads(open('$out/c3_${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', $rep, 'ez', e['value'], e.get('ms_per_search'))" >> $out/summary.txt
  done
done
timeout -k 10 300 python bench.py > $out/bench.json 2>&1
cat $out/summary.txt
