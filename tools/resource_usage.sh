#!/bin/bash
# Per-kernel register / spill / LDS report of liblzmcts (compiler remarks), filtered by a pattern.
# usage: tools/resource_usage.sh [kernel-name-regex]
set -euo pipefail
pat=${1:-search_}
out=${TMPDIR:-/tmp}/lzm_ru.txt
/opt/rocm/bin/hipcc -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -fPIC -shared --offload-arch=gfx950 \
  -Rpass-analysis=kernel-resource-usage -o ${TMPDIR:-/tmp}/lzm_ru.so lightzero_amd/csrc/lzm_kernels.hip 2> "$out" || true
python3 - "$out" "$pat" <<'PY'
import re, sys
txt = open(sys.argv[1]).read().splitlines()
pat = re.compile(sys.argv[2])
cur = None
for line in txt:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        show = bool(pat.search(cur))
        if show:
            print(cur)
        continue
    if cur and show and re.search(r"(VGPRs|AGPRs|Spill|LDS Size|Occupancy|ScratchSize)", line):
        print("   ", line.split("remark:")[-1].strip())
PY
