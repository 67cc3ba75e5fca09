"""Build the HIP engine in-tree: dmclock_amd/libdmclock_gpu.so (gfx950)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "libdmclock_gpu.so")
SOURCES = [os.path.join(HERE, "csrc", "dmc_engine.hip")]
# every source and header under csrc/ plus the C-ABI header
DEPS = SOURCES + sorted(
    os.path.join(HERE, "csrc", f) for f in os.listdir(os.path.join(HERE, "csrc"))
    if f.endswith((".h", ".hip"))) + [os.path.join(ROOT, "include", "dmclock_gpu.h")]

HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               # exact IEEE double tag arithmetic: no FMA contraction
               "-ffp-contract=off",
               # (strict aliasing holds: every whole-word access to memory
               # declared with other types goes through ld_as / st_as,
               # csrc/dmc_device.h)
               "-Wall", "-Wno-unused-function"]


def up_to_date():
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(d) <= t for d in DEPS)


def build(force=False, verbose=True):
    if not force and up_to_date():
        return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    tmp = LIB + ".tmp"
    cmd = [hipcc] + HIPCC_FLAGS + ["-o", tmp] + SOURCES
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    os.replace(tmp, LIB)  # (atomic: a snapshot never sees a half-written library)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
