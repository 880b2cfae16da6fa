"""Compiled-scene cache: one rank compiles the scene (SBVH build, ~36 s and a
3.5 GB host scene at C3 size), writes every array of its ctl_scene_desc to one
file, and the other ranks of the node map that file instead of compiling
again.  The mapped pages are shared between the ranks (the page cache of
/dev/shm), so N ranks hold one host copy instead of N.

File layout: 8-byte magic, 8-byte header length, a JSON header (the desc's
fixed part as hex bytes, and per array field its offset and byte count), then
the arrays, each at a 4 KiB-aligned offset.  A desc read back has the same
scalars and array bytes as the one written; its pointers point into the map.
Nothing here is loaded from files this process did not expect: the header is
JSON and the arrays are raw bytes of the layouts in _abi.py."""
import ctypes as C
import json
import mmap
import os

import numpy as np

from . import _abi

MAGIC = b"CTLSCN01"

# pointer field -> (element type, element count of a desc)
_ARRAYS = {
    "tri_data": (_abi.TriangleData, lambda d: d.n_tri_data),
    "woop_tris": (_abi.WoopTri, lambda d: d.n_woop_tris),
    "bvh_nodes": (_abi.BVHNode, lambda d: d.n_bvh_nodes),
    "tri_indices": (C.c_uint32, lambda d: d.n_tri_indices),
    "materials": (_abi.Material, lambda d: d.n_materials),
    "meshes": (_abi.KernelMesh, lambda d: d.n_meshes),
    "nodes": (_abi.Node, lambda d: d.n_nodes),
    "scene_bvh_nodes": (_abi.BVHNode, lambda d: d.n_scene_bvh_nodes),
    "node_xf": (_abi.Float4x4, lambda d: d.n_nodes),
    "node_inv_xf": (_abi.Float4x4, lambda d: d.n_nodes),
    "lights": (_abi.Light, lambda d: d.n_lights),
    "light_tris": (_abi.LightTri, lambda d: d.n_light_tris),
    "light_tri_cdf": (C.c_float, lambda d: d.n_light_tri_cdf),
    "textures": (_abi.Texture, lambda d: d.n_textures),
    "tex_data": (C.c_uint32, lambda d: d.n_tex_data),
    "env": (_abi.EnvLight, lambda d: 1),
    "env_data": (C.c_float, lambda d: d.n_env_data),
    "mesh_boxes": (C.c_float, lambda d: 6 * d.n_meshes),
    "anim_vertices": (_abi.AnimVertex, lambda d: d.n_anim_vertices),
    "anim_triangles": (C.c_uint32, lambda d: 3 * d.n_anim_triangles),
    "anim_meshes": (_abi.AnimMesh, lambda d: d.n_anim_meshes),
}


def _addr(p):
    return C.cast(p, C.c_void_p).value or 0


def save(desc, path):
    """Writes desc to `path` (atomically: a temporary name, then a rename)."""
    layout = {}
    off = 0
    for name, (et, count) in _ARRAYS.items():
        nbytes = C.sizeof(et) * int(count(desc)) if _addr(getattr(desc, name)) else 0
        off = (off + 4095) & ~4095
        layout[name] = [off, nbytes]
        off += nbytes
    header = json.dumps({"desc": bytes(desc).hex(), "arrays": layout, "desc_size": C.sizeof(desc)}).encode()
    base = (16 + len(header) + 4095) & ~4095
    tmp = f"{path}.tmp{os.getpid()}"
    with open(tmp, "wb") as f:
        f.write(MAGIC + len(header).to_bytes(8, "little") + header)
        for name, (o, nbytes) in layout.items():
            if nbytes:
                f.seek(base + o)
                f.write(memoryview((C.c_char * nbytes).from_address(_addr(getattr(desc, name)))).cast("B"))
        f.truncate(base + off)
    os.replace(tmp, path)
    return base + off


class Cached:
    """A desc whose arrays live in a read-only map of a cache file."""

    def __init__(self, path):
        with open(path, "rb") as f:
            head = f.read(16)
            if head[:8] != MAGIC:
                raise ValueError(f"{path}: not a scene cache")
            hlen = int.from_bytes(head[8:16], "little")
            h = json.loads(f.read(hlen).decode())
            if h["desc_size"] != C.sizeof(_abi.SceneDesc):
                raise ValueError(f"{path}: written for another SceneDesc layout")
            self._map = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
        base = (16 + hlen + 4095) & ~4095
        self.desc = _abi.SceneDesc.from_buffer_copy(bytes.fromhex(h["desc"]))
        buf = memoryview(self._map)
        self._arrays = []
        for name, (o, nbytes) in h["arrays"].items():
            et, _ = _ARRAYS[name]
            if nbytes == 0:
                setattr(self.desc, name, C.POINTER(et)())
                continue
            if base + o + nbytes > len(self._map):
                raise ValueError(f"{path}: array {name} past the end of the file")
            a = np.frombuffer(buf, dtype=np.uint8, count=nbytes, offset=base + o)
            self._arrays.append(a)
            setattr(self.desc, name, C.cast(C.c_void_p(a.ctypes.data), C.POINTER(et)))

    def close(self):
        self._arrays.clear()
        self.desc = None
        self._map.close()


def load(path):
    """The desc of a cache file (keep the returned object alive while the desc is used)."""
    return Cached(path)
