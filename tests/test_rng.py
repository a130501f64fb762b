"""Counter-based RNG (include/rt_rng.h): Random123 Philox4x32-10 known answers,
exact 24-bit uniforms and the rand.Intn replacement."""
import ctypes as C
import os
import shutil
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

KAT = [  # Random123 kat_vectors, philox4x32 10 rounds
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
]


@pytest.fixture(scope="module")
def rnglib(tmp_path_factory):
    if shutil.which("gcc") is None:
        pytest.skip("no C compiler")
    d = tmp_path_factory.mktemp("rng")
    src = d / "rng.c"
    src.write_text('#include "rt_rng.h"\n'
                   "void philox(const unsigned* c, const unsigned* k, unsigned* o){"
                   "rt_u32x4 r = rt_philox4x32_10(c[0],c[1],c[2],c[3],k[0],k[1]);"
                   "for(int i=0;i<4;++i) o[i]=r.v[i];}\n"
                   "unsigned pick(unsigned x, unsigned n){return rt_pick(x,n);}\n"
                   "unsigned resid(unsigned x, unsigned n){return rt_pick_residual(x,n);}\n"
                   "float unitf(unsigned x){return rt_unit_f(x);}\n"
                   "double unitd(unsigned x){return rt_unit_d(x);}\n")
    so = d / "librng.so"
    subprocess.run(["gcc", "-O2", "-shared", "-fPIC", "-I", os.path.join(REPO, "include"),
                    str(src), "-o", str(so)], check=True)
    L = C.CDLL(str(so))
    L.pick.restype = C.c_uint
    L.resid.restype = C.c_uint
    L.unitf.restype = C.c_float
    L.unitd.restype = C.c_double
    return L


@pytest.mark.parametrize("ctr,key,expect", KAT)
def test_philox_kat(rnglib, ctr, key, expect):
    o = (C.c_uint * 4)()
    rnglib.philox((C.c_uint * 4)(*ctr), (C.c_uint * 2)(*key), o)
    assert tuple(o) == expect


def test_uniforms_exact_in_float_and_double(rnglib):
    for x in [0, 1, 255, 256, 0x7fffffff, 0xffffffff, 0x12345678]:
        f, d = rnglib.unitf(x), rnglib.unitd(x)
        assert f == d  # 24-bit mantissa: identical in fp32 and fp64
        assert 0.0 <= d < 1.0
    assert rnglib.unitd(0xffffffff) == 1.0 - 2.0 ** -24


def test_pick_matches_floor_and_nesting(rnglib):
    rng = np.random.default_rng(0)
    for n in [1, 2, 3, 7, 100, 12345]:
        for x in rng.integers(0, 2 ** 32, 200, dtype=np.uint64):
            x = int(x)
            u = (x >> 8) / 2.0 ** 24
            p = rnglib.pick(x, n)
            assert p == int(np.floor(u * n)) and p < n
            # the residual is the fractional part of u*n, again a 24-bit uniform
            r = rnglib.resid(x, n)
            assert (r >> 8) == ((x >> 8) * n) & 0xFFFFFF
