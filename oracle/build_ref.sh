#!/usr/bin/env bash
# Builds the REFERENCE ctree (LightZero ctree_muzero / ctree_efficientzero) from the
# sources where they lie under /root/reference, into oracle/_ref/ only.
# Test infrastructure: used to pin the CPU restatement (oracle/lz_oracle.c) and to
# generate tests/golden/*.npz. Never shipped, never on the product path.
#
# Recipe: cython --cplus on the reference .pyx (output redirected
# into oracle/_ref/build), then g++ with Python's own extension flags (-O2 -fwrapv
# -DNDEBUG, no -mfma) plus -Wl,--wrap=gettimeofday so that the time-seeded srand()
# inside cbatch_traverse (common_lib/utils.cpp:25) becomes controllable.
set -euo pipefail
REF=${LZ_REFERENCE:-/root/reference}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT=$HERE/_ref
CT=$REF/lzero/mcts/ctree
if [ ! -d "$CT" ]; then
  echo "build_ref: $CT not present; skipping reference build" >&2
  exit 0
fi
mkdir -p "$OUT/build"
PYINC=$(python3 -c "import sysconfig;print(sysconfig.get_paths()['include'])")
EXT=$(python3 -c "import sysconfig;print(sysconfig.get_config_var('EXT_SUFFIX'))")
CXXFLAGS="-DNDEBUG -g0 -fwrapv -O2 -fPIC -shared -std=c++11 -w"
gcc -O2 -fPIC -c "$HERE/ref_time_hook.c" -o "$OUT/build/ref_time_hook.o"
for pair in ctree_muzero:mz_tree ctree_efficientzero:ez_tree; do
  d=${pair%%:*}; m=${pair##*:}
  cython --cplus -3 -I "$CT/$d" -o "$OUT/build/$m.cpp" "$CT/$d/$m.pyx"
  g++ $CXXFLAGS -I"$PYINC" -I"$CT/$d" "$OUT/build/$m.cpp" "$OUT/build/ref_time_hook.o" \
      -Wl,--wrap=gettimeofday -o "$OUT/$m$EXT"
done
# AlphaZero tree: pybind11 from pip; the reference's own sources, unchanged.
AZ=$CT/ctree_alphazero
if [ -f "$AZ/mcts_alphazero.cpp" ] && python3 -c "import pybind11" 2>/dev/null; then
  g++ -O2 -shared -std=c++17 -fPIC -w $(python3 -m pybind11 --includes) -I"$AZ" "$AZ/mcts_alphazero.cpp" \
      -o "$OUT/mcts_alphazero$EXT"
fi
echo "build_ref: built $(ls "$OUT"/*"$EXT" | xargs -n1 basename | tr '\n' ' ')"
