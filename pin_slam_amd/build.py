"""Build the gfx950 shared library in-tree: pin_slam_amd/libpin_slam_amd.so.

hipcc cross-compiles for gfx950 without a GPU, so this runs in the build
container; the resulting .so travels to the GPU box with the repo snapshot.
"""
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB = os.path.join(HERE, "libpin_slam_amd.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

FLAGS = [
    "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
    # every elementwise op rounds like the reference's unfused ATen ops; FMAs are explicit
    "-ffp-contract=off",
    "-Wall", "-Wno-unused-function",
]


def sources():
    return sorted(glob.glob(os.path.join(HERE, "csrc", "*.hip")))


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = sources() + glob.glob(os.path.join(HERE, "csrc", "*.h")) + [os.path.join(ROOT, "include", "pin_slam_amd.h")]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, extra=(), out: str = None) -> str:
    """Compile every csrc/*.hip into one shared library (``out`` defaults to the in-tree LIB;
    ``extra`` adds compiler flags, e.g. -D switches for experiment variants)."""
    out = out or LIB
    if out == LIB and not force and not _stale():
        return LIB
    cmd = [HIPCC, *FLAGS, *extra, "-I", os.path.join(ROOT, "include"), "-I", os.path.join(HERE, "csrc"),
           *sources(), "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(LIB)
