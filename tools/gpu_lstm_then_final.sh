# GPU: the LSTM gate GEMM on split-fp16 (lightzero_amd/liblzm_varL.so): its conv / config 3 / divergence tests
# and an interleaved Pong EZ A/B against the default library; when the tests pass and the variant is faster,
# it becomes the library (copied over liblzmcts.so, the same file the local tree then takes). Then the round's
# closing set runs (on whichever library won). A test failure (pytest exit 1) keeps the default library; any
# other failure (fault, abort, time limit) ends the call. usage: bash tools/gpu_lstm_then_final.sh
out=gpurun_out/r05ah
rc=0
bash tools/gpu_lstm_check.sh $out || rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "LSTM check ended with $rc: stopping"; exit $rc; fi
if [ $rc -eq 0 ]; then
  python3 - <<'PY' > $out/decision.txt
import json, glob
def t(v):
    return [json.loads(open(f).read().strip().splitlines()[-1])["ms_per_search"] for f in sorted(glob.glob(f"gpurun_out/r05ah/c3_{v}_*.json"))]
cur, L = t("cur"), t("L")
print("swap" if max(L) < min(cur) else "keep", cur, L)
PY
else
  echo "keep (tests failed)" > $out/decision.txt
fi
cat $out/decision.txt
if grep -q '^swap' $out/decision.txt; then cp lightzero_amd/liblzm_varL.so lightzero_amd/liblzmcts.so; fi
set -e
bash tools/gpu_final_r05.sh a && bash tools/gpu_final_r05.sh b
