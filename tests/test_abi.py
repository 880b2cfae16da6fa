"""The C-ABI library loads and exports every symbol include/ctl_trace.h
declares; the ctypes layouts match the reference sizes.  No GPU calls."""
import ctypes as C
import os
import re

import pytest

import cudatracerlib_amd._abi as abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "ctl_trace.h")).read()
    return sorted(set(re.findall(r"CTL_API\s+[\w\s\*]+?\b(ctl_\w+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(abi.LIB_PATH)
    names = declared_symbols()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(n for n, _, _ in abi.SYMBOLS) == names


def test_abi_version():
    # round 5: ctl_occluded; the 8-wide tree's flag, arrays and ctl_host_w8_tree gone
    assert abi.load().ctl_abi_version() == 4 == abi.ABI_VERSION


def test_load_refuses_another_abi_version(tmp_path, monkeypatch):
    """A library reporting another CTL_ABI_VERSION (stale build, CTL_LIB variant)
    is refused before anything binds to its struct layouts."""
    import shutil
    copy = tmp_path / "libctl_trace.so"   # another path: load() does not return its cached handle
    shutil.copy(abi.LIB_PATH, copy)
    monkeypatch.setattr(abi, "ABI_VERSION", abi.ABI_VERSION + 1)
    with pytest.raises(RuntimeError, match="CTL_ABI_VERSION"):
        abi.load(str(copy))



def test_reference_layout_sizes():
    assert C.sizeof(abi.BVHNode) == 64        # BVHNodeData
    assert C.sizeof(abi.WoopTri) == 48        # TriIntersectorData
    assert C.sizeof(abi.TriangleData) == 32   # TriangleData (EXT_TRI)
    assert C.sizeof(abi.KernelMesh) == 20     # KernelMesh
    assert C.sizeof(abi.Node) == 24           # Node
    assert C.sizeof(abi.Ray) == 32            # traversalRay
    assert C.sizeof(abi.Hit) == 16            # traversalResult
    assert C.sizeof(abi.Pixel) == 28          # PixelData
    assert C.sizeof(abi.LightTri) == 64       # ShapeSet::triData
    assert C.sizeof(abi.Material) == 80       # flattened Material + BSDF parameters
    assert C.sizeof(abi.Texture) == 380       # ImageTexture + KernelMIPMap
    assert C.sizeof(abi.PixelVariance) == 44  # PixelVarianceInfo
    assert C.sizeof(abi.Light) == 48          # flattened DiffuseLight / InfiniteLight header
    assert C.sizeof(abi.EnvLight) == 112      # InfiniteLight (+ m_worldTransform rotation)


# ctypes mirror <-> include/ctl_trace.h: every field offset and struct size as
# the C compiler lays them out (gcc on a generated probe, no GPU needed)
_LAYOUT_STRUCTS = [("ctl_scene_desc", "SceneDesc"), ("ctl_light", "Light"), ("ctl_env_light", "EnvLight"),
                   ("ctl_texture", "Texture"), ("ctl_material", "Material"), ("ctl_camera", "Camera")]


_C_FIELD = {("ctl_texture", "mapping"): "m11"}   # the mirror packs m11..m23 as one array


def test_struct_layouts_match_header(tmp_path):
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "ctl_trace.h"', 'int main(void) {']
    expect = []
    for cname, pname in _LAYOUT_STRUCTS:
        py = getattr(abi, pname)
        lines.append(f'printf("%zu\\n", sizeof({cname}));')
        expect.append(C.sizeof(py))
        for f in py._fields_:
            cfield = _C_FIELD.get((cname, f[0]), f[0])
            lines.append(f'printf("%zu\\n", offsetof({cname}, {cfield}));')
            expect.append(getattr(py, f[0]).offset)
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert got == expect


def test_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        return
    L = abi.load()
    assert not L.ctl_create(0)
    assert L.ctl_last_error(None)
