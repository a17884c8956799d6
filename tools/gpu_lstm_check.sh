# GPU: the conv / config 3 GPU tests on lightzero_amd/liblzm_varL.so (the LSTM gate GEMM on split-fp16),
# then the Pong EZ search bench against the default library, interleaved twice. usage: bash ... OUT
set -e
out=$1
mkdir -p $out
LZM_LIB=lightzero_amd/liblzm_varL.so timeout -k 10 600 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_config3.py tests/test_gpu_divergence.py > $out/t.log 2>&1
for rep in 1 2; do
  for v in cur L; do
    lib=lightzero_amd/liblzmcts.so
    [ "$v" != cur ] && lib=lightzero_amd/liblzm_var$v.so
    LZM_LIB=$lib timeout -k 10 200 python tools/conv_bench.py --kind ez --searches 10 > $out/c3_${v}_$rep.json 2>&1
    python3 -c "import json;e=json.loads(open('$out/c3_${v}_$rep.json').read().strip().splitlines()[-1]);print('$v', $rep, 'ez', e['value'], e.get('ms_per_search'))" >> $out/summary.txt
  done
done
cat $out/summary.txt
