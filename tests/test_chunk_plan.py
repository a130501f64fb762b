"""CPU model of the fused kernel's chunk plan (rt_render.hip render_impl, rt_path.h
chunk_pixel / chunk_ids, rt_render.hip k_resolve): every sample of every
pixel belongs to exactly one chunk, the chunks k_resolve sums for a pixel are exactly the
chunks whose ids map to it, and the two-phase plan (a first phase of K-sample chunks, then a
tail of K2-sample chunks) changes only how samples are grouped.  Pixel sums are exact integer
sums, so any grouping gives the same image (tests/test_render_gpu.py checks that on the GPU)."""
import itertools

import pytest


def plan(npix, ss, K, gpix, tail_frac=0, tail_k=None):
    """Host side: (K, K2, S1, cpp1, cpp2, n1, n_chunks), as render_impl computes them."""
    S1, K2 = ss, K
    if tail_frac > 1 and K >= 8:
        K2 = max(4, tail_k if tail_k else K // 4)
        s1 = (ss * (tail_frac - 1) // tail_frac) // K * K
        if 0 < s1 < ss and K2 < K:
            S1 = s1
        else:
            K2 = K
    cpp1 = S1 // K + (1 if S1 == ss and ss % K else 0)
    cpp2 = (ss - S1 + K2 - 1) // K2 if S1 < ss else 0
    assert npix % gpix == 0
    return dict(K=K, K2=K2, S1=S1, cpp1=cpp1, cpp2=cpp2, n1=npix * cpp1,
                n=npix * (cpp1 + cpp2), gch=gpix * cpp1, gch2=max(1, gpix * cpp2), gpix=gpix, ss=ss)


def chunk_ids(p, c):
    """Device side: chunk id -> (local pixel, first sample, sample count)."""
    tail = c >= p["n1"]
    cc = c - p["n1"] if tail else c
    g = p["gch2"] if tail else p["gch"]
    q, r = divmod(cc, g)
    sub, rr = divmod(r, p["gpix"])
    lp = q * p["gpix"] + rr
    s0 = p["S1"] + sub * p["K2"] if tail else sub * p["K"]
    cnt = min(p["K2"], p["ss"] - s0) if tail else min(p["K"], p["S1"] - s0)
    return lp, s0, cnt


def resolve_chunks(p, lp):
    """k_resolve: the chunk records it sums for local pixel lp."""
    q, r = divmod(lp, p["gpix"])
    out = []
    for ph in (0, 1):
        gch = p["gch2"] if ph else p["gch"]
        cpp = 0 if ph and p["S1"] >= p["ss"] else gch // p["gpix"]  # no tail: no second loop
        base = (p["n1"] if ph else 0) + q * gch + r
        out += [base + sb * p["gpix"] for sb in range(cpp)]
    return out


CASES = [(npix, gpix, ss, K, tf)
         for (npix, gpix), ss, K, tf in itertools.product(
             [(12, 4), (30, 10), (7, 7), (5, 1)], [1, 9, 16, 484, 1024], [4, 8, 16, 32], [0, 4, 8])]


@pytest.mark.parametrize("npix,gpix,ss,K,tf", CASES)
def test_every_sample_once_and_resolve_matches(npix, gpix, ss, K, tf):
    K = min(K, ss)
    p = plan(npix, ss, K, gpix, tf)
    seen = [[0] * ss for _ in range(npix)]
    owner = {}
    for c in range(p["n"]):
        lp, s0, cnt = chunk_ids(p, c)
        assert 0 <= lp < npix and cnt >= 1
        for s in range(s0, s0 + cnt):
            seen[lp][s] += 1
        owner.setdefault(lp, []).append(c)
    assert all(v == 1 for row in seen for v in row)
    for lp in range(npix):
        assert sorted(resolve_chunks(p, lp)) == sorted(owner[lp])
    if tf > 1 and p["S1"] < ss:
        # the tail is the last chunk ids, made of the shorter chunks
        assert all(chunk_ids(p, c)[1] >= p["S1"] for c in range(p["n1"], p["n"]))
        assert p["K2"] < p["K"]
