# GPU: fused LSTM kernel timing with parts removed (diagnostic builds via LZM_LIB; results invalid)
set -e
out=gpurun_out/${1:-lsd}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python tools/lstm_bench.py > $out/base.txt 2>&1
for d in ${DIAGS:-1 2 3}; do
  LZM_LIB=lightzero_amd/liblzm_lsd$d.so timeout -k 10 120 python tools/lstm_bench.py --no-check > $out/diag$d.txt 2>&1
done
