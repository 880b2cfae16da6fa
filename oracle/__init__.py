"""ctypes binding of the oracle (TEST INFRASTRUCTURE ONLY).

The oracle is a CPU restatement of the reference algorithm (oracle/oracle.cpp).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module; the product (cudatracerlib_amd) never does.
"""
import ctypes as C
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
# ORACLE_LIB: another build of the same sources (the sanitizer build, tools/san_tests.sh)
LIB = os.environ.get("ORACLE_LIB") or os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

TIE_FIRST_FOUND = 0   # the reference's binary visit order (the reference semantics)
TRAVERSE_WIDE = 2     # the product's 4-wide per-ray order over trees registered with oracle_set_wide
# any-hit shadow query culling: tmax - eps (round 4) / tmax / none / tmax + slab slack (the product's)
CULL_AT_ACCEPT, CULL_AT_TMAX, CULL_AT_INF, CULL_SLAB = 0, 1, 2, 3


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    from cudatracerlib_amd._abi import SceneDesc, Camera, PTParams, Pixel, PrimParams
    L = C.CDLL(LIB)
    vp = C.c_void_p
    sig = {
        "oracle_set_wide": (None, [C.POINTER(SceneDesc), vp, C.c_uint64, vp, C.c_uint32, vp, C.c_uint64]),
        "oracle_woop_set": (None, [vp, vp, vp, vp]),
        "oracle_woop_get": (None, [vp, vp, vp, vp]),
        "oracle_xorwow_uniforms": (None, [C.c_uint64, C.c_uint64, C.c_uint64, vp]),
        "oracle_xorwow_raw": (None, [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint64, vp]),
        "oracle_sampler_tables": (None, [C.c_uint64, C.c_uint32, C.c_uint32, vp, vp]),
        "oracle_sampler_draws": (None, [vp, vp, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, vp, C.c_uint32, vp]),
        "oracle_camera": (None, [vp, vp, vp, C.c_float, C.c_float, C.c_float, C.c_uint32, C.c_uint32,
                                 C.POINTER(Camera)]),
        "oracle_trace": (None, [C.POINTER(SceneDesc), C.c_int64, vp, C.c_int32, C.c_int32, vp, vp, vp, vp, vp, vp,
                                C.c_int32]),
        "oracle_intersect": (None, [C.POINTER(SceneDesc), C.c_int64, vp, vp, C.c_int32, C.c_int32, C.c_int32]),
        "oracle_occluded": (None, [C.POINTER(SceneDesc), C.c_int64, vp, vp, C.c_int32, C.c_int32, C.c_int32,
                                   C.c_int32]),
        "oracle_brute_force": (None, [C.POINTER(SceneDesc), C.c_int64, vp, vp, vp, C.c_int32]),
        "oracle_render_pass": (C.c_uint64, [C.POINTER(SceneDesc), C.POINTER(PTParams), C.c_uint64, vp, C.c_int32,
                                            C.c_int32, C.c_uint32, vp]),
        "oracle_camera_rays": (None, [C.POINTER(SceneDesc), C.c_uint64, vp]),
        "oracle_prim_pass": (C.c_uint64, [C.POINTER(SceneDesc), C.POINTER(PrimParams), C.c_uint64, vp, vp, C.c_int32,
                                          C.c_int32]),
        "oracle_animate": (None, [C.POINTER(SceneDesc), C.c_uint32, vp, vp, C.c_float, vp, vp, vp, vp, vp, vp]),
        "oracle_scene_set_transform": (None, [C.POINTER(SceneDesc), vp, vp, vp, C.c_uint32, vp]),
        "oracle_wpt_render_pass": (C.c_uint64, [C.POINTER(SceneDesc), C.c_int32, C.c_int32, C.c_int32, C.c_uint32,
                                                C.c_uint64, vp, C.c_int32, C.c_int32]),
        "oracle_image_resolve": (None, [vp, C.c_uint32, C.c_uint32, C.c_float, vp]),
        "oracle_variance_add_pass": (None, [vp, C.c_uint32, C.c_uint32, C.c_float, C.c_uint32, vp, vp]),
        "oracle_variance_stats": (None, [vp, C.c_uint64, vp, vp, vp]),
        "oracle_triangle_data_set": (None, [vp, C.c_uint8, vp, vp, vp]),
        "oracle_light_tri": (None, [vp, vp, vp, vp, vp, vp]),
        "oracle_matrix_inverse": (None, [vp, vp]),
        "oracle_env_tables": (None, [vp, vp, vp, vp]),
        "oracle_env_sample": (None, [C.POINTER(SceneDesc), C.c_uint64, vp, vp]),
        "oracle_env_eval": (None, [C.POINTER(SceneDesc), C.c_uint64, vp, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def ptr(a):
    return a.ctypes.data_as(C.c_void_p)
