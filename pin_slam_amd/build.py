"""Build the gfx950 shared library in-tree: pin_slam_amd/libpin_slam_amd.so.

hipcc cross-compiles for gfx950 without a GPU, so this runs in the build
container; the resulting .so travels to the GPU box with the repo snapshot.
"""
import glob
import os
import shutil
import subprocess
import sys
import tempfile

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
    # one object per source, compiled in parallel (objects outside the tree), then one link
    objdir = tempfile.mkdtemp(prefix="pin_slam_amd_obj_")
    inc = ["-I", os.path.join(ROOT, "include"), "-I", os.path.join(HERE, "csrc")]
    try:
        procs = []
        objs = []
        for src in sources():
            obj = os.path.join(objdir, os.path.basename(src) + ".o")
            cmd = [HIPCC, *[f for f in FLAGS if f != "-shared"], *extra, *inc, "-c", src, "-o", obj]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            procs.append((cmd, subprocess.Popen(cmd)))
            objs.append(obj)
        for cmd, p in procs:
            if p.wait() != 0:
                raise subprocess.CalledProcessError(p.returncode, cmd)
        subprocess.run([HIPCC, *FLAGS, *objs, "-o", out + ".tmp"], check=True)
    finally:
        shutil.rmtree(objdir, ignore_errors=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(LIB)
