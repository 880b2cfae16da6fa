"""Traversal stack bound (host logic, no GPU): ctl_host_bvh_stack_bound, the
check ctl_scene_upload runs before a scene reaches the device.  The bound is
the deepest stack the traversal in device/traverse.h can build on a tree:
1 sentinel + the largest sum of (children - 1) along a root-to-node path."""
import ctypes as C
import struct

import pytest

SENT = 0x76543210


def as_f(i):
    return struct.unpack("<f", struct.pack("<i", i))[0]


def chain(ctl, depth, leaf_first=True):
    """Binary BVHNodeData chain: node i has a leaf child and node i+1 (the
    last node: a leaf and the sentinel).  Boxes are unit boxes."""
    nodes = (ctl._abi.BVHNode * depth)()
    for i in range(depth):
        v = [0.0, 1.0, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0, 0.0, 0.0, 0.0, 0.0]
        nxt = (i + 1) * 4 if i + 1 < depth else SENT
        leaf = ~i
        a, b = (leaf, nxt) if leaf_first else (nxt, leaf)
        v[12], v[13] = as_f(a), as_f(b)
        nodes[i].v[:] = v
    return nodes


@pytest.mark.parametrize("depth", [1, 2, 7, 40, 200])
def test_chain_bound(ctl, depth):
    b, w = ctl.bvh_stack_bound(chain(ctl, depth))
    # every node but the last pushes one entry (its two children are used);
    # the last node has one used child (sentinel excluded)
    assert b == 1 + (depth - 1)
    # a chain collapses into wide nodes of 3 leaves + 1 inner child
    assert 1 <= w <= 1 + 3 * (b - 1)


def test_balanced_tree_bound(ctl):
    """Complete binary tree of 2^k - 1 inner nodes: bound = 1 + k (binary) and
    at most that for the collapsed 4-wide tree."""
    k = 10
    n = 2 ** k - 1
    nodes = (ctl._abi.BVHNode * n)()
    for i in range(n):
        l, r = 2 * i + 1, 2 * i + 2
        cl = l * 4 if l < n else ~i
        cr = r * 4 if r < n else ~(i + n)
        v = [0.0, 1.0] * 6 + [as_f(cl), as_f(cr), 0.0, 0.0]
        nodes[i].v[:] = v
    b, w = ctl.bvh_stack_bound(nodes)
    assert b == 1 + k
    # a wide node covers at least one binary level and pushes at most 3 (the
    # collapse opens the largest child first, so on equal boxes it opens
    # unevenly and the wide stack can be deeper than the binary one)
    assert 1 + k // 2 <= w <= 1 + 3 * (b - 1)


def test_deep_trees(ctl):
    b, w = ctl.bvh_stack_bound(chain(ctl, 700))
    assert b == 700 and w > 128          # far past the device stack: upload refuses it
    with pytest.raises(ctl.CTLError):   # deeper than the 4-wide collapse takes
        ctl.bvh_stack_bound(chain(ctl, 2000))


@pytest.mark.parametrize("bad", ["cycle", "range", "misaligned"])
def test_malformed_tree_is_refused(ctl, bad):
    nodes = chain(ctl, 8)
    v = list(nodes[5].v)
    v[13] = as_f({"cycle": 2 * 4, "range": 100 * 4, "misaligned": 6 * 4 + 1}[bad])
    nodes[5].v[:] = v
    with pytest.raises(ctl.CTLError):
        ctl.bvh_stack_bound(nodes)


@pytest.mark.parametrize("config,scale", [(1, 1.0), (2, 0.25), (3, 0.004), (5, 0.003)])
def test_compiled_scenes_fit_the_device_stack(ctl, config, scale):
    """Every mesh tree the compiler emits for the configs fits the 128-entry
    device stack with room to spare."""
    hs = ctl.HostScene().generate(config, scale, 64, 64)   # owns the desc's arrays
    d = hs.compile()
    for m in range(d.n_meshes):
        first = d.meshes[m].bvh_node_offset // 4
        n = d.n_bvh_nodes - first
        arr = C.cast(C.addressof(d.bvh_nodes.contents) + first * 64, C.POINTER(ctl._abi.BVHNode * n)).contents
        b, w = ctl.bvh_stack_bound(arr)
        assert b < 100 and w < 100, (m, b, w)
