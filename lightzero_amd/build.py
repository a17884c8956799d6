"""Builds liblzmcts.so in-tree for gfx950 (hipcc). Invoked by __graft_entry__.build()."""
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("LZM_OFFLOAD_ARCH", "gfx950")
# -ffp-contract=off: no fused multiply-add anywhere in the tree kernels, so every fp32
# expression rounds like the reference's SSE build; division and sqrt stay IEEE (HIP default).
# -fno-slp-vectorize: no v_pk_fma_f32 pairing in the fused search's dense layers — its operand
# pairs cost ~3 v_mov each (measured: ~370 -> ~75 moves per network step).
FLAGS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-fPIC", "-shared", "-Wall",
         f"--offload-arch={ARCH}"]
SOURCES = [os.path.join(HERE, "csrc", "lzm_kernels.hip")]
DEPS = SOURCES + sorted(glob.glob(os.path.join(HERE, "csrc", "*.h"))) + [
    os.path.join(REPO, "include", "lzmcts.h")]
OUT = os.path.join(HERE, "liblzmcts.so")


def needs_build():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(d) > t for d in DEPS)


def build(force=False, verbose=True):
    if not force and not needs_build():
        return OUT
    cmd = [HIPCC] + FLAGS + ["-o", OUT] + SOURCES
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
