"""CPU checks of the native boundary and host logic (no GPU calls)."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from oracle import pin_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "pin_slam_amd.h")).read()
    return sorted(set(re.findall(r"^(?:int|int64_t) (pin_\w+)\(", hdr, flags=re.M)))


def test_library_exports_every_declared_symbol():
    from pin_slam_amd import _lib
    lib = _lib.load()
    decl = declared_symbols()
    assert decl, "no entry points parsed from the header"
    for name in decl:
        assert hasattr(lib, name), f"{name} declared in include/pin_slam_amd.h but not exported"
    assert sorted(_lib.exported_symbols()) == decl, "ctypes signature table out of sync with the header"


STRUCTS = ["PinHash", "PinPoints", "PinGridDims", "PinGrid", "PinMlp", "PinRegParams", "PinTrainCfg",
           "PinTrainState", "PinAdamStep", "PinMapArrays", "PinSampleCfg", "PinRegIter", "PinRowArray"]


def test_struct_layouts_match_header(tmp_path):
    """sizeof / offsetof of every ABI struct, compiled from include/pin_slam_amd.h with gcc,
    against the ctypes mirrors in pin_slam_amd/_lib.py."""
    import shutil
    import subprocess
    from pin_slam_amd import _lib
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "pin_slam_amd.h"', "int main(void) {"]
    for name in STRUCTS:
        lines.append(f'printf("{name} sizeof %zu\\n", sizeof({name}));')
        for field, _ in getattr(_lib, name)._fields_:
            lines.append(f'printf("{name} {field} %zu\\n", offsetof({name}, {field}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    got = {(a, b): int(c) for a, b, c in (line.split() for line in out if line)}
    for name in STRUCTS:
        cls = getattr(_lib, name)
        assert got[(name, "sizeof")] == ctypes.sizeof(cls), name
        for field, _ in cls._fields_:
            assert got[(name, field)] == getattr(cls, field).offset, (name, field)
    # every struct the header declares is mirrored
    hdr = open(os.path.join(ROOT, "include", "pin_slam_amd.h")).read()
    assert sorted(re.findall(r"^} (Pin\w+);", hdr, re.M)) == sorted(STRUCTS)


def test_header_constants_match_bindings():
    from pin_slam_amd import _lib
    hdr = open(os.path.join(ROOT, "include", "pin_slam_amd.h")).read()
    val = lambda name: int(re.search(r"#define %s (\d+)" % name, hdr).group(1))  # noqa: E731
    assert val("PIN_MLP_PACK_BYTES") == _lib.MLP_PACK_BYTES
    assert val("PIN_ORDER_STATE_BYTES") == __import__("pin_slam_amd.query", fromlist=["x"]).ORDER_STATE_BYTES


def test_neighbor_offsets_host(golden):
    from pin_slam_amd.neural_points import neighbor_offsets
    z = golden("neighborhoods")
    for key in [k for k in z if k.endswith("_dx")]:
        c, a = key.split("_")[:2]
        got = neighbor_offsets(int(c[1:]), int(a[1:]) / 10).numpy()
        np.testing.assert_array_equal(got, z[key])


def test_hash_slots_host_matches_oracle():
    from pin_slam_amd.neural_points import hash_slots
    rng = np.random.default_rng(0)
    p = rng.uniform(-500, 500, (10000, 3)).astype(np.float32)
    for B in (1 << 17, int(5e7)):
        got = hash_slots(torch.from_numpy(p), 0.3, B).numpy()
        np.testing.assert_array_equal(got, O.hash_slots(O.voxel_coords(p, 0.3), B))


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    from pin_slam_amd import _lib
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    try:
        _lib.load()
    except RuntimeError as e:
        assert "no fallback" in str(e)
    else:
        raise AssertionError("load() must raise when the native library is missing")


def test_cpu_tensors_are_rejected():
    import pin_slam_amd as P
    nm = P.NeuralPoints(P.Config(device="cpu", buffer_size=1 << 10))
    try:
        nm.query_feature(torch.zeros(4, 3))
    except RuntimeError as e:
        assert "ROCm device" in str(e)
    else:
        raise AssertionError("CPU tensors must not silently run a fallback")


def test_argument_errors_before_any_device_work():
    """Bad arguments come back as PIN_ERR_ARG / PIN_ERR_UNSUPPORTED before anything touches the
    device (so these run without a GPU)."""
    from pin_slam_amd import _lib
    lib = _lib.load()
    m = _lib.PinMlp()
    assert lib.pin_mlp_pack(None, None, None) == -1
    assert lib.pin_mlp_pack(ctypes.byref(m), None, None) == -1           # NULL weights
    m.W1 = m.b1 = m.W2 = m.b2 = 16
    assert lib.pin_mlp_pack(ctypes.byref(m), ctypes.c_void_p(8), None) == -1   # packed not 16-B aligned
    st = _lib.PinAdamStep(grad_stride=4)
    assert lib.pin_adam_rows(None, None, None, None, None, 0, ctypes.byref(st), None) == -3   # stride != 8
    cfg = _lib.PinTrainCfg(n_main=-1, decimation=1)
    assert lib.pin_train_rows(None, ctypes.byref(cfg), None, None) == -1
