"""The C-ABI library loads and exports every symbol include/ctl_trace.h
declares; the ctypes layouts match the reference sizes.  No GPU calls."""
import ctypes as C
import os
import re

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
    assert abi.load().ctl_abi_version() == 1


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


def test_create_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        return
    L = abi.load()
    assert not L.ctl_create(0)
    assert L.ctl_last_error(None)
