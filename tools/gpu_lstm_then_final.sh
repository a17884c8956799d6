# GPU: the LSTM gate GEMM on split-fp16 (lightzero_amd/liblzm_varL.so): its conv / config 3 / divergence tests
# and an interleaved Pong EZ A/B against the default library; when the tests pass and the variant is faster,
# it becomes the library (copied over liblzmcts.so, the same file the local tree then takes) and the round's
# closing set runs on it. usage: bash tools/gpu_lstm_then_final.sh
set -e
out=gpurun_out/r05ah
bash tools/gpu_lstm_check.sh $out
python3 - <<'PY' > $out/decision.txt
import json, glob
def t(v):
    return [json.loads(open(f).read().strip().splitlines()[-1])["ms_per_search"] for f in sorted(glob.glob(f"gpurun_out/r05ah/c3_{v}_*.json"))]
cur, L = t("cur"), t("L")
print("swap" if max(L) < min(cur) else "keep", cur, L)
PY
cat $out/decision.txt
if grep -q '^swap' $out/decision.txt; then
  cp lightzero_amd/liblzm_varL.so lightzero_amd/liblzmcts.so
  rm -rf gpurun_out/final_r05
  bash tools/gpu_final_r05.sh a && bash tools/gpu_final_r05.sh b
fi
