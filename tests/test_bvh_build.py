"""The alternative BVH4 builder: a Morton-ordered binary tree
(PLOC clustering or an LBVH radix tree) collapsed with collectChildren's rule, or by the
surface-area cost model (IZPI_BVH_SAH), into the reference's BVH4Node format.

CPU side (here): the oracle's sequential restatement of the builder (oracle_lbvh4)
yields valid BVH4 trees (the invariants of bvh4_test.go:13-83,453-496 that do not
depend on the reference's split rule), the host's primitive boxes equal the oracle's,
and a scene traversed through that tree finds the same closest hits as through the
reference tree. GPU side (tests/test_gpu_parity.py): the GPU builder's arrays equal
oracle_lbvh4's bit for bit, and renders on its tree equal the oracle's on the same tree.
"""
import numpy as np
import pytest

from izpi_amd import _native as N
from izpi_amd import configs
from izpi_amd.scene import HostScene
from oracle import oracle as O

F32_MAX = np.float32(3.4028234663852886e38)


def node_view(nodes):
    nodes = np.ascontiguousarray(nodes, np.uint8)
    f = nodes[:, :96].copy().view(np.float32).reshape(-1, 6, 4)   # min x/y/z, max x/y/z per slot
    i = nodes[:, 96:].copy().view(np.int32).reshape(-1, 2, 4)     # child, prim_count per slot
    return f, i[:, 0], i[:, 1]


def check_tree(nodes, order, boxes, leaf_max=4):
    n = len(boxes)
    f, child, count = node_view(nodes)
    assert sorted(order.tolist()) == list(range(n))
    covered = np.zeros(n, np.int32)
    parent_slot = {}
    for k in range(len(nodes)):
        if count[k, 0] > 0:  # leaf: slot 0 only (bvh4.go:736-760)
            s, c = child[k, 0], count[k, 0]
            assert 1 <= c <= leaf_max and (child[k, 1:] == -1).all() and (count[k, 1:] == 0).all()
            covered[s:s + c] += 1
            pb = boxes[order[s:s + c]]
            lo, hi = pb[:, :3].min(0), pb[:, 3:].max(0)
            assert (f[k, :3, 0].astype(np.float64) <= lo).all() and (f[k, 3:, 0].astype(np.float64) >= hi).all()
            if k in parent_slot:  # the leaf box is bit-identical to its parent's slot box (A10)
                p, sl = parent_slot[k]
                assert f[k, :, 0].tobytes() == f[p, :, sl].tobytes()
            continue
        assert (count[k] == 0).all()
        for sl in range(4):
            c = child[k, sl]
            if c == -1:
                assert (f[k, :, sl] == F32_MAX).all()
                continue
            assert k < c < len(nodes)
            parent_slot[c] = (k, sl)
    assert (covered == 1).all()
    # every slot box holds the boxes of its subtree's primitives
    def prims(k):
        if count[k, 0] > 0:
            return order[child[k, 0]:child[k, 0] + count[k, 0]].tolist()
        return sum((prims(c) for c in child[k] if c != -1), [])
    for k in range(min(len(nodes), 64)):
        if count[k, 0] > 0:
            continue
        for sl in range(4):
            c = child[k, sl]
            if c == -1:
                continue
            pb = boxes[prims(c)]
            assert (f[k, :3, sl].astype(np.float64) <= pb[:, :3].min(0)).all()
            assert (f[k, 3:, sl].astype(np.float64) >= pb[:, 3:].max(0)).all()


def test_host_prim_boxes_equal_oracle():
    for scene in (configs.cornell_dragon(1.0, n=12), configs.cornell_glass_spectral(1.0)):
        h = HostScene(scene, 1.0)
        o = O.OracleScene(scene, 1.0)
        assert h.prim_boxes().tobytes() == o.prim_boxes().tobytes()


@pytest.mark.parametrize("method", [N.BVH_LBVH, N.BVH_PLOC, N.BVH_PLOC_SAH])
@pytest.mark.parametrize("n_side", [1, 3, 24])
def test_lbvh4_tree_invariants(n_side, method):
    scene = configs.cornell_dragon(1.0, n=n_side)
    boxes = HostScene(scene, 1.0, skip_bvh=True).prim_boxes()
    for lm in (3, 4):
        nodes, order = O.lbvh4(boxes, lm, method)
        check_tree(nodes, order, boxes, leaf_max=lm)


@pytest.mark.parametrize("method", [N.BVH_LBVH, N.BVH_PLOC, N.BVH_PLOC_SAH])
def test_lbvh4_small_and_degenerate_inputs(method):
    rng = np.random.default_rng(2)
    for n in (1, 2, 4, 5, 17):
        lo = rng.uniform(0, 10, (n, 3))
        boxes = np.concatenate([lo, lo + rng.uniform(0.1, 1, (n, 3))], 1)
        nodes, order = O.lbvh4(boxes, 4, method)
        check_tree(nodes, order, boxes)
        if n <= 4:
            assert len(nodes) == 1
    same = np.tile([1.0, 1.0, 1.0, 2.0, 2.0, 2.0], (37, 1))  # one Morton code, equal boxes
    nodes, order = O.lbvh4(same, 4, method)
    check_tree(nodes, order, same)
    assert order.tolist() == list(range(37))  # split by position / paired by position
    f, child, count = node_view(nodes)
    assert len(nodes) < 40  # balanced, not a chain
    for lm in (1, 2, 3):
        nodes, order = O.lbvh4(boxes, lm, method)
        check_tree(nodes, order, boxes, leaf_max=lm)


def test_lbvh4_scene_finds_the_reference_closest_hits():
    """Through the linear BVH the oracle finds the same closest-hit distances as through
    the reference tree (only equal-t ties may pick another primitive)."""
    scene = configs.cornell_dragon(1.0, n=24)
    ref = O.OracleScene(scene, 1.0)
    alt = O.OracleScene(scene, 1.0)
    nodes, order = O.lbvh4(alt.prim_boxes(), 3)
    alt.set_bvh(nodes, order)
    rng = np.random.default_rng(7)
    n = 4000
    o = np.column_stack([rng.uniform(5, 95, n), rng.uniform(5, 95, n), rng.uniform(5, 95, n)])
    d = rng.normal(size=(n, 3))
    rays = np.column_stack([o, d, np.full(n, 0.001), np.full(n, np.finfo(np.float64).max)])
    a, b = ref.trace(rays), alt.trace(rays)
    ta = np.array([h.t if h.hit else np.inf for h in a])
    tb = np.array([h.t if h.hit else np.inf for h in b])
    assert (ta == tb).all()
    assert sum(h.prim_ref != g.prim_ref for h, g in zip(a, b)) <= n // 1000


def sah_cost(nodes, cn=1.0, cl=0.5, ct=1.0):
    """Surface-area cost of a BVH4 under the builder's model: each wide node's visit (cn)
    and each leaf's visit and primitive tests (cl + ct per primitive), weighted by the
    half area of the node's box (its slot box in the parent; the root: its slots' union)."""
    f, child, count = node_view(nodes)
    def ha(lo, hi):
        d = hi.astype(np.float64) - lo.astype(np.float64)
        return d[0] * d[1] + d[1] * d[2] + d[2] * d[0]
    used = child[0] != -1
    total = cn * ha(f[0, :3, used].min(0), f[0, 3:, used].max(0)) if count[0, 0] == 0 else 0.0
    for k in range(len(nodes)):
        if count[k, 0] > 0:
            continue
        for sl in range(4):
            c = child[k, sl]
            if c == -1:
                continue
            a = ha(f[k, :3, sl], f[k, 3:, sl])
            total += a * (cl + ct * count[c, 0]) if count[c, 0] > 0 else a * cn
    return total


@pytest.mark.parametrize("lm", [2, 3, 4])
def test_sah_collapse_costs_less(lm):
    """IZPI_BVH_SAH picks the collapse of least surface-area cost over the same PLOC binary
    tree: its cost under that model is below the greedy collectChildren collapse's, and it
    keeps the same leaf order (the collapse only regroups the binary tree's subtrees)."""
    scene = configs.cornell_dragon(1.0, n=24)
    boxes = HostScene(scene, 1.0, skip_bvh=True).prim_boxes()
    g_nodes, g_order = O.lbvh4(boxes, lm, N.BVH_PLOC)
    s_nodes, s_order = O.lbvh4(boxes, lm, N.BVH_PLOC_SAH)
    assert (g_order == s_order).all()
    check_tree(s_nodes, s_order, boxes, leaf_max=lm)
    assert sah_cost(s_nodes) < sah_cost(g_nodes)


def test_set_bvh_validates():
    scene = configs.cornell_dragon(1.0, n=3)
    h = HostScene(scene, 1.0, skip_bvh=True)
    assert h.desc.num_nodes == 0
    nodes, order = O.lbvh4(h.prim_boxes())
    h.set_bvh(nodes, order)
    assert h.desc.num_nodes == len(nodes) and 0 < h.stack_bound <= 64
    bad = order.copy()
    bad[0] = bad[1]
    with pytest.raises(RuntimeError, match="permutation"):
        h.set_bvh(nodes, bad)


@pytest.mark.parametrize("scene_name", ["dragon", "glass", "degenerate"])
def test_quantized_boxes_contain_the_exact_ones(scene_name):
    """oracle.quantize_bvh4 (IZPI_SCENE_QUANTIZED_BVH restated): the tree stays a valid BVH4
    over the same primitives, every decoded slot box contains the exact one,
    a leaf node's box is its parent slot's decoded box, and the boxes grow by little (mean extent
    growth of the leaf boxes < 5% on the dragon)."""
    if scene_name == "degenerate":
        boxes = np.tile([1.0, 1.0, 1.0, 2.0, 2.0, 2.0], (40, 1))
        boxes[::2, 3:] = boxes[::2, :3]  # flat boxes: zero extent on every axis
    else:
        scene = configs.cornell_dragon(1.0, n=40) if scene_name == "dragon" else configs.cornell_glass_spectral(1.0)
        boxes = HostScene(scene, 1.0, skip_bvh=True).prim_boxes()
    nodes, order = O.lbvh4(boxes, 3, N.BVH_PLOC_SAH)
    q, applied = O.quantize_bvh4(nodes)
    assert applied
    check_tree(q, order, boxes, leaf_max=3)
    f0, child, count = node_view(nodes)
    f1, child1, count1 = node_view(q)
    assert (child == child1).all() and (count == count1).all()
    inner = count[:, 0] == 0
    valid = (child != -1) & inner[:, None]
    lo0, hi0, lo1, hi1 = f0[:, :3], f0[:, 3:], f1[:, :3], f1[:, 3:]
    v = np.repeat(valid[:, None, :], 3, 1)
    assert (lo1[v] <= lo0[v]).all() and (hi1[v] >= hi0[v]).all()
    for k in np.flatnonzero(inner):  # leaves take their parent slot's decoded box
        for sl in range(4):
            c = child[k, sl]
            if c >= 0 and count[c, 0] > 0:
                assert f1[c, :, 0].tobytes() == f1[k, :, sl].tobytes()
    if scene_name == "dragon":
        leaf = count[:, 0] > 0
        ext0 = (f0[leaf, 3:, 0] - f0[leaf, :3, 0]).astype(np.float64)
        ext1 = (f1[leaf, 3:, 0] - f1[leaf, :3, 0]).astype(np.float64)
        assert ext1.sum() / ext0.sum() < 1.05, ext1.sum() / ext0.sum()


def test_quantized_tree_finds_the_same_closest_hits():
    """Traversing the decoded boxes finds the closest hits of the exact ones (the oracle's
    trace through both trees: equal t and primitive except at exact ties)."""
    scene = configs.cornell_dragon(1.0, n=40)
    o = O.OracleScene(scene, aspect_override=1.0)
    nodes, order = O.lbvh4(o.prim_boxes(), 3, N.BVH_PLOC_SAH)
    rng = np.random.default_rng(7)
    n = 3000
    rays = np.zeros((n, 8))
    rays[:, :3] = rng.uniform([5, 5, -50], [95, 95, 95], (n, 3))
    rays[:, 3:6] = rng.normal(size=(n, 3))
    rays[:, 6], rays[:, 7] = 0.001, np.finfo(np.float64).max
    o.set_bvh(nodes, order)
    a = o.trace(rays)
    o.set_bvh(O.quantize_bvh4(nodes)[0], order)
    b = o.trace(rays)
    o.close()
    same = sum(bytes(a[i])[:72] == bytes(b[i])[:72] and a[i].prim_ref == b[i].prim_ref for i in range(n))
    assert same == n
