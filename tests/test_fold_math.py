"""The backward clamp fold of rayColor (camera.go:316, :328-330) as the fused kernel
computes it (rt_path.h shade_core + WStack::fold_max), checked in fp64 against the
reference's step-by-step recursion on random paths.  CPU only: this pins the algebra
(telescoped scale, merged dominated vertices, the media kernels' cascade), not fp32.

Reference (per clamp vertex k, from the last one back):
    v_k = clamp(w_k * v_k+1),  clamp(c) = c * M / I(c) if I(c) = r+g+b > M else c
Kernel: the pending weight of the latest clamp vertex is held apart; on a new clamp
vertex it is pushed, or -- when it lies in [0, 1]^3 -- multiplied into the stack top
(and, cascading, the top folded down while it lies in [0, 1]^3); at the end
    P = pend * L, maxI = I(P), walk the stack back: P = e * P, maxI = max(maxI, I(P)),
    result = P * min(1, M / maxI).
"""
import numpy as np
import pytest

M = 1.5


def reference(ws, L):
    v = np.array(L, np.float64)
    for w in reversed(ws):
        v = w * v
        i = v.sum()
        if i > M:
            v = v * (M / i)
    return v


def kernel(ws, L, cascade, merge_ok=True):
    """merge_ok: DevScene.merge_ok -- every colour, albedo and the background >= 0
    (rt_render.hip upload_scene / render_impl); with it off every vertex is pushed."""
    stack, pend = [], None
    for w in ws:
        if pend is not None:
            merge = merge_ok and len(stack) > 0 and np.all(pend >= 0) and np.all(pend <= 1)
            if merge:
                stack[-1] = stack[-1] * pend
                while cascade and len(stack) >= 2 and np.all(stack[-1] >= 0) and \
                        np.all(stack[-1] <= 1):
                    top = stack.pop()
                    stack[-1] = stack[-1] * top
            else:
                stack.append(pend)
        pend = np.array(w, np.float64)
    v = pend * np.array(L, np.float64)
    max_i = v.sum()
    for e in reversed(stack):
        v = e * v
        max_i = max(max_i, v.sum())
    return v * (M / max_i) if max_i > M else v, len(stack)


@pytest.mark.parametrize("cascade", [False, True])
def test_merged_fold_equals_stepwise_clamps(cascade):
    rng = np.random.default_rng(7)
    depth_saved = 0
    for trial in range(4000):
        n = int(rng.integers(1, 41))
        # weights like att * spdf / pdf: albedo in [0, 1) times a ratio in (0, 2]
        ws = [rng.random(3) * rng.uniform(0.05, 2.0) for _ in range(n)]
        if trial % 7 == 0:
            ws = [w * 0.5 for w in ws]  # mostly dominated vertices
        L = rng.random(3) * rng.choice([0.5, 4.0, 15.0])
        got, depth = kernel(ws, L, cascade)
        want = reference(ws, L)
        np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-15)
        depth_saved += (n - 1) - depth
    assert depth_saved > 0  # the merge did shorten stacks


def test_zero_and_boundary_weights():
    L = [3.0, 2.0, 1.0]
    for ws in ([np.zeros(3), np.ones(3) * 2.0, np.ones(3)],
               [np.ones(3), np.ones(3), np.ones(3)],
               [np.array([1.0, 0.0, 1.0]), np.array([2.0, 0.5, 0.1])]):
        for cascade in (False, True):
            got, _ = kernel(ws, L, cascade)
            np.testing.assert_allclose(got, reference(ws, L), rtol=1e-12, atol=1e-15)


def test_negative_radiance_needs_the_unmerged_fold():
    """A negative background or colour makes the suffix products signed: a weight in
    [0, 1]^3 can then raise I(P) (P = (10, -9, 0), w = (1, 0, 0): I 1 -> 10), so the
    merge would skip a clamp the reference applies.  Scenes with any negative value run
    with merge_ok = 0 (rt_render.hip), and the telescoped fold alone is exact for any
    sign: the clamp scales are positive, and a vertex with I <= M never clamps."""
    ws = [np.array([0.1, 1.0, 1.0]), np.array([1.0, 0.0, 0.0]), np.array([1.0, 1.0, 1.0])]
    L = np.array([10.0, -9.0, 0.0])
    merged, _ = kernel(ws, L, cascade=False, merge_ok=True)
    assert not np.allclose(merged, reference(ws, L))  # the case the flag exists for
    rng = np.random.default_rng(11)
    for trial in range(4000):
        n = int(rng.integers(1, 30))
        ws = [rng.uniform(-0.5, 1.0, 3) * rng.uniform(0.05, 2.0) for _ in range(n)]
        if trial % 3 == 0:  # non-negative weights, mixed-sign radiance
            ws = [np.abs(w) for w in ws]
        L = rng.uniform(-1.0, 1.0, 3) * rng.choice([0.5, 4.0, 15.0])
        for cascade in (False, True):
            got, depth = kernel(ws, L, cascade, merge_ok=False)
            assert depth == max(0, n - 1)
            np.testing.assert_allclose(got, reference(ws, L), rtol=1e-10, atol=1e-12)
