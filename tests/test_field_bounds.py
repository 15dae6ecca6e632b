"""CPU: the device arithmetic headers (firedancer_amd/csrc/*_dev.h) compiled for
the host and driven at the documented limb bounds against Python big ints.
This pins the radix-2^25.5 bound bookkeeping (R / M bounds, no 64-bit column
overflow) and the scalar / SHA helpers the kernel uses."""
import ctypes
import hashlib
import os
import random
import struct
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 2**255 - 19
LL = 2**252 + 27742317777372353535851937790883648493
POS = [0, 26, 51, 77, 102, 128, 153, 179, 204, 230]
R_E, R_O = 2**26 + 2**11, 2**25 + 2**16
M_E, M_O = 3 * 2**26 + 2**13, 3 * 2**25 + 2**18
F_E, F_O = 5 * 2**26 + 3 * 2**11, 5 * 2**25 + 3 * 2**16   # "F": uncarried first operand (fd_f25519_dev.h)


@pytest.fixture(scope="module")
def lib():
    out = os.path.join(REPO, "tests", "_build")
    os.makedirs(out, exist_ok=True)
    so = os.path.join(out, "field_host_check.so")
    src = os.path.join(REPO, "tests", "csrc", "field_host_check.cpp")
    subprocess.check_call(["g++", "-O2", "-shared", "-fPIC", "-o", so, src])
    return ctypes.CDLL(so)


def val(l):
    return sum(x << POS[i] for i, x in enumerate(l))


def arr(l, t=ctypes.c_uint32):
    return (t * len(l))(*l)


def limbs_at(be, bo, mode, rng):
    return [(be if i % 2 == 0 else bo) if mode == "max" else rng.randrange(0, (be if i % 2 == 0 else bo) + 1)
            for i in range(10)]


def in_R(h):
    return all(x <= (R_E if i % 2 == 0 else R_O) for i, x in enumerate(h))


def test_mul_sq_at_bounds(lib):
    rng = random.Random(1)
    for it in range(3000):
        mode = "max" if it < 20 else "rand"
        f = limbs_at(M_E, M_O, mode, rng); g = limbs_at(M_E, M_O, mode, rng)
        h = (ctypes.c_uint32 * 10)(); lib.t_mul(h, arr(f), arr(g)); h = list(h)
        assert val(h) % P == val(f) * val(g) % P and in_R(h)
        h = (ctypes.c_uint32 * 10)(); lib.t_sq(h, arr(f)); h = list(h)
        assert val(h) % P == val(f) ** 2 % P and in_R(h)


def test_mul_uncarried_first_operand(lib):
    """fe_mul( h, F, M ): the doubling's Fn = 2ZZ + XX + 2p - YY and the mixed
    addition's F = 2Z + 2p - TT go in uncarried as the first operand
    (fd_curve25519_dev.h ge_dbl / ge_madd); the product stays exact and in R."""
    rng = random.Random(7)
    for it in range(3000):
        mode = "max" if it < 20 else "rand"
        f = limbs_at(F_E, F_O, mode, rng); g = limbs_at(M_E, M_O, mode, rng)
        h = (ctypes.c_uint32 * 10)(); lib.t_mul(h, arr(f), arr(g)); h = list(h)
        assert val(h) % P == val(f) * val(g) % P and in_R(h)
    # the operands as the formulas build them, at their own maxima
    r = [R_E if i % 2 == 0 else R_O for i in range(10)]
    two_p = [2 * (2**26 - 19)] + [2 * (2**26 - 1) if i % 2 == 0 else 2 * (2**25 - 1) for i in range(1, 10)]
    fn = [3 * r[i] + two_p[i] for i in range(10)]            # 2ZZ + XX + 2p - 0
    assert all(x <= (F_E if i % 2 == 0 else F_O) for i, x in enumerate(fn))
    # ge_dbl forms Fn as 2 ZZ + (4p - G), G = YY - XX + 2p: 4p - G stays
    # nonnegative per limb at G's largest value (YY = R, XX = 0), and the sum
    # is limbwise the same 2ZZ + XX - YY + 2p
    sd = (ctypes.c_uint32 * 10)(); lib.t_sub4p(sd, arr([r[i] + two_p[i] for i in range(10)])); sd = list(sd)
    assert all(0 <= v < 2**31 for v in sd)
    for it in range(2000):
        zz = limbs_at(R_E, R_O, "max" if it < 5 else "rand", rng)
        xx = limbs_at(R_E, R_O, "max" if it < 5 else "rand", rng)
        yy = limbs_at(R_E, R_O, "max" if it < 5 else "rand", rng)
        g = [yy[i] + two_p[i] - xx[i] for i in range(10)]
        sd = (ctypes.c_uint32 * 10)(); lib.t_sub4p(sd, arr(g)); sd = list(sd)
        fn2 = [2 * zz[i] + sd[i] for i in range(10)]
        assert fn2 == [2 * zz[i] + xx[i] + two_p[i] - yy[i] for i in range(10)]
        assert all(x <= (F_E if i % 2 == 0 else F_O) for i, x in enumerate(fn2))
    fm = [2 * r[i] + two_p[i] for i in range(10)]            # 2Z + 2p - 0
    assert all(x <= (F_E if i % 2 == 0 else F_O) for i, x in enumerate(fm))


def test_sq_seed_doubling_e(lib):
    """ge_dbl's E = (X+Y)^2 - (XX+YY): H = XX + YY left uncarried (2R, a
    first operand only), the square seeded with 4p - H per column
    (fe_sq_seed, fd_curve25519_dev.h) -- exact, and E comes out in R."""
    rng = random.Random(11)
    r = [R_E if i % 2 == 0 else R_O for i in range(10)]
    for it in range(3000):
        mode = "max" if it < 20 else "rand"
        x = limbs_at(R_E, R_O, mode, rng); y = limbs_at(R_E, R_O, mode, rng)
        hh = [x[i] + y[i] for i in range(10)]                     # XX + YY, both R
        assert all(v <= (M_E if i % 2 == 0 else M_O) for i, v in enumerate(hh))
        sd = (ctypes.c_uint32 * 10)(); lib.t_sub4p(sd, arr(hh)); sd = list(sd)
        assert all(0 <= v < 2**31 for v in sd) and val(sd) % P == (-val(hh)) % P
        f = limbs_at(M_E, M_O, mode, rng)                          # X + Y: M
        h = (ctypes.c_uint32 * 10)(); lib.t_sq_seed(h, arr(f), arr(sd)); h = list(h)
        assert val(h) % P == (val(f) ** 2 - val(hh)) % P and in_R(h)
    # the largest H the formula forms still leaves 4p - H nonnegative
    sd = (ctypes.c_uint32 * 10)(); lib.t_sub4p(sd, arr([2 * v for v in r])); assert all(v < 2**31 for v in sd)


def test_sub_carry_canon(lib):
    rng = random.Random(2)
    for it in range(3000):
        mode = "max" if it < 20 else "rand"
        a = limbs_at(R_E, R_O, mode, rng); b = limbs_at(R_E, R_O, mode, rng)
        h = (ctypes.c_uint32 * 10)(); lib.t_sub(h, arr(a), arr(b)); h = list(h)
        assert val(h) % P == (val(a) - val(b)) % P
        assert all(x <= (M_E if i % 2 == 0 else M_O) for i, x in enumerate(h))
        c = [rng.randrange(0, 2**31) for _ in range(10)] if mode == "rand" else [2**31 - 1] * 10
        h = (ctypes.c_uint32 * 10)(); lib.t_carry(h, arr(c)); h = list(h)
        assert val(h) % P == val(c) % P and in_R(h)
        f = limbs_at(M_E, M_O, mode, rng)
        o = (ctypes.c_uint32 * 8)(); lib.t_tobytes(o, arr(f))
        assert sum(x << (32 * i) for i, x in enumerate(o)) == val(f) % P
    for v in [0, 1, P - 1, P, P + 1, P + 18, 2**255 - 1]:
        lim = [(v >> POS[i]) & ((1 << (26 if i % 2 == 0 else 25)) - 1) for i in range(10)]
        o = (ctypes.c_uint32 * 8)(); lib.t_tobytes(o, arr(lim))
        assert sum(x << (32 * i) for i, x in enumerate(o)) == v % P


def test_frombytes_not_reduced(lib):
    rng = random.Random(3)
    for _ in range(500):
        w = [rng.randrange(0, 2**32) for _ in range(8)]
        h = (ctypes.c_uint32 * 10)(); lib.t_frombytes(h, arr(w))
        assert val(list(h)) == sum(x << (32 * i) for i, x in enumerate(w)) % 2**255   # bit 255 dropped only


def test_pow22523(lib):
    rng = random.Random(4)
    for _ in range(20):
        f = limbs_at(R_E, R_O, "rand", rng)
        h = (ctypes.c_uint32 * 10)(); lib.t_pow22523(h, arr(f))
        assert val(list(h)) % P == pow(val(f), 2**252 - 3, P)


def test_scalar_reduce_and_check(lib):
    rng = random.Random(5)
    edge = [0, 1, LL, LL - 1, LL + 1, 2**512 - 1, LL * 3, 2**252, 2**511, LL * 2**259]
    for it in range(20000):
        x = edge[it] if it < len(edge) else rng.getrandbits(512)
        r = (ctypes.c_uint32 * 8)(); lib.t_sc_reduce(r, arr([(x >> (32 * i)) & 0xffffffff for i in range(16)]))
        assert sum(v << (32 * i) for i, v in enumerate(r)) == x % LL
    lib.t_sc_lt_l.restype = ctypes.c_int
    for s in [LL - 1, LL, LL + 1, 0, 2**256 - 1, 2**253, LL - 2**200, 2**252]:
        assert lib.t_sc_lt_l(arr([(s >> (32 * i)) & 0xffffffff for i in range(8)])) == (s < LL)


def test_recoding(lib):
    rng = random.Random(6)
    for it in range(3000):
        s = rng.getrandbits(253) if it else LL - 1
        w = arr([(s >> (32 * i)) & 0xffffffff for i in range(8)])
        o4 = (ctypes.c_uint8 * 64)(); lib.t_recode4(o4, w)
        assert sum((d - 8) * 16**i for i, d in enumerate(o4)) == s and all(0 <= d <= 16 for d in o4)
        o8 = (ctypes.c_uint8 * 32)(); lib.t_recode8(o8, w)
        assert sum((d - 128) * 256**i for i, d in enumerate(o8)) == s


def test_sha512_block(lib):
    iv = [0x6a09e667f3bcc908, 0xbb67ae8584caa73b, 0x3c6ef372fe94f82b, 0xa54ff53a5f1d36f1,
          0x510e527fade682d1, 0x9b05688c2b3e6c1f, 0x1f83d9abfb41bd6b, 0x5be0cd19137e2179]
    h = arr(iv, ctypes.c_uint64)
    w = arr([0x8000000000000000] + [0] * 15, ctypes.c_uint64)
    lib.t_sha_block(h, w)
    assert b"".join(struct.pack(">Q", v) for v in h) == hashlib.sha512(b"").digest()


def test_lattice_short_vector_host(lib):
    """fd_lattice_dev.h compiled for the host: on random and structured k the
    search returns u = v k (mod 8l), v odd, 0 < v < l (what makes
    [v]([S]B - [k]A - R) == O equivalent to the reference's equation) with
    |u|, |v| around 2^128 (what the chain's window count is sized for; the
    bounds of the device test, test_gpu_parity.py)."""
    rng = random.Random(9)
    ks = [rng.randrange(LL) for _ in range(20000)]
    ks += [0, 1, 2, 3, LL - 1, LL - 2, 2**128 - 1, 2**128, 2**128 + 1, 2**127, 2**200, 2**252,
           (8 * LL // 3) % LL, (8 * LL // 5) % LL, 2**64, 12345]
    ks += [rng.randrange(1 << rng.randrange(1, 253)) for _ in range(2000)]
    n8, bits = 8 * LL, []
    u, v, un = (ctypes.c_uint32 * 8)(), (ctypes.c_uint32 * 8)(), ctypes.c_int()
    for k in ks:
        it = lib.t_lattice(arr([(k >> (32 * j)) & 0xffffffff for j in range(8)]), u, v, ctypes.byref(un))
        assert it < 1024, k                                      # not the (k, 1) fallback
        uu = val32(u) * (-1 if un.value else 1)
        vv = val32(v)
        assert vv % 2 == 1 and 0 < vv < LL and (uu - vv * k) % n8 == 0, (k, uu, vv)
        if k and k % LL:
            assert lat_euclid_check(k, uu, vv, n8), (k, uu, vv)
        bits.append(max(abs(uu).bit_length(), vv.bit_length()))
    assert max(bits[:20000]) <= 140 and sorted(bits[:20000])[19800] <= 131


def lat_euclid_check(k, u, v, n8):
    """The search's output is the one the exact extended Euclid on (8l, k)
    gives: at the first remainder r_i < 2^128, (u, v) = (r_i, t_i) up to sign
    when t_i is odd, else (r_{i-1} - j r_i, t_{i-1} - j t_i) for some j >= 0
    (fd_lattice_dev.h).  Pins every quotient of the Lehmer rounds, not only
    the lattice relation."""
    r0, t0, r1, t1 = n8, 0, k, 1
    while r1 >= 2**128:
        q = r0 // r1
        r0, r1, t0, t1 = r1, r0 - q * r1, t1, t0 - q * t1
    if t1 % 2:
        return (u, v) == ((r1, t1) if t1 > 0 else (-r1, -t1))
    j, rem = divmod(v - abs(t0), abs(t1))
    return rem == 0 and j >= 0 and u == (r0 - j * r1) * (1 if t0 > 0 else -1)


def val32(w):
    return sum(int(x) << (32 * i) for i, x in enumerate(w))


def test_comb_digits(lib):
    """The fixed-base comb's signed 23-bit digits (fd_scalar_dev.h comb_bias /
    comb_digit, and the cached kernel's shifting form): sum d_k 2^(23 k) = w,
    |d_k| <= 2^22 for k < 10 and 0 <= d_10 <= 2^22 (the table's 2^22 + 1
    entries per position), for random w < l and the edges."""
    rng = random.Random(23)
    ws = [rng.randrange(LL) for _ in range(20000)] + [0, 1, LL - 1, LL - 2, 2**252 - 1, 2**252, 2**230,
                                                     2**230 - 1, 2**22, 2**22 - 1, 2**23 - 1, 2**23]
    ws += [sum(rng.choice([0, 2**22 - 1, 2**22, 2**23 - 1]) << (23 * k) for k in range(10)) % LL for _ in range(2000)]
    ws += [(LL - 1) - sum(rng.choice([0, 1, 2**22]) << (23 * k) for k in range(10)) for _ in range(2000)]
    d = (ctypes.c_int * 11)()
    for w in ws:
        lib.t_comb_digits(d, arr([(w >> (32 * j)) & 0xffffffff for j in range(8)]))
        dd = list(d)
        assert 0x7fffffff not in dd, w
        assert sum(x << (23 * k) for k, x in enumerate(dd)) == w, w
        assert all(-2**22 <= x < 2**22 for x in dd[:10]) and 0 <= dd[10] <= 2**22, (w, dd)


N_1 = 2**26 - 1    # fe_sq_neg / fe_finish_neg: limb 1 taken from 2^26 - 1


def in_N(h):
    return all(0 <= x <= ((2**26 - 1) if i % 2 == 0 else (2**25 - 1)) for i, x in enumerate(h) if i != 1) and 0 <= h[1] <= N_1


def test_sq_neg_complement(lib):
    """fe_sq_neg: -f^2 in complement form (column 0 seeded with 18 + 2^51, every
    limb taken from its mask, limb 1 from 2^26 - 1): exact mod p at the M bounds,
    limbs never negative."""
    rng = random.Random(21)
    for it in range(4000):
        mode = "max" if it < 20 else "rand"
        f = limbs_at(M_E, M_O, mode, rng)
        if it % 7 == 3:
            f = [0] * 10; f[rng.randrange(10)] = rng.randrange(0, 3)     # tiny values: the seed carries through
        h = (ctypes.c_uint32 * 10)(); lib.t_sq_neg(h, arr(f)); h = list(h)
        assert val(h) % P == (-val(f) ** 2) % P and in_N(h), (f, h)


def test_dbl_operands_at_bounds(lib):
    """ge_dbl's negated operands: E' = (XX + YY) + (-(X+Y)^2) (2R + N, a second
    operand) and G' = XX + 2p - YY; X' = Fn E' and T' = H E' stay exact and in R
    with Fn at the F bound and E' at its own largest limbs."""
    rng = random.Random(23)
    r = [R_E if i % 2 == 0 else R_O for i in range(10)]
    n = [(2**26 - 1) if i % 2 == 0 else (2**25 - 1) for i in range(10)]; n[1] = N_1
    ep_max = [2 * r[i] + n[i] for i in range(10)]
    assert all(19 * x < 2**32 for x in ep_max)
    for it in range(3000):
        mode = "max" if it < 20 else "rand"
        ep = [x if mode == "max" else rng.randrange(0, x + 1) for x in ep_max]
        f = limbs_at(F_E, F_O, mode, rng); hh = [2 * x if mode == "max" else rng.randrange(0, 2 * x + 1) for x in r]
        h = (ctypes.c_uint32 * 10)(); lib.t_mul(h, arr(f), arr(ep)); h = list(h)
        assert val(h) % P == val(f) * val(ep) % P and in_R(h)
        h = (ctypes.c_uint32 * 10)(); lib.t_mul(h, arr(hh), arr(ep)); h = list(h)
        assert val(h) % P == val(hh) * val(ep) % P and in_R(h)


def test_pair_ops_and_cneg(lib):
    """fe_add / fe_lshl1_add / fe_sub as limb-pair (64-bit) operations equal the
    limbwise ones at the F bound (no carry between the halves); fe_cneg is
    2p - a or a."""
    rng = random.Random(29)
    two_p = [2 * (2**26 - 19)] + [2 * (2**26 - 1) if i % 2 == 0 else 2 * (2**25 - 1) for i in range(1, 10)]
    for it in range(2000):
        mode = "max" if it < 10 else "rand"
        a = limbs_at(F_E, F_O, mode, rng); b = limbs_at(M_E, M_O, mode, rng)
        h = (ctypes.c_uint32 * 10)(); lib.t_add(h, arr(a), arr(b)); assert list(h) == [a[i] + b[i] for i in range(10)]
        z = limbs_at(R_E, R_O, mode, rng)
        h = (ctypes.c_uint32 * 10)(); lib.t_lshl1_add(h, arr(z), arr(b)); assert list(h) == [2 * z[i] + b[i] for i in range(10)]
        x = limbs_at(R_E, R_O, mode, rng); y = limbs_at(R_E, R_O, mode, rng)
        h = (ctypes.c_uint32 * 10)(); lib.t_sub(h, arr(x), arr(y)); assert list(h) == [x[i] + two_p[i] - y[i] for i in range(10)]
        for neg in (0, 1):
            h = (ctypes.c_uint32 * 10)(); lib.t_cneg(h, arr(x), neg)
            assert list(h) == ([two_p[i] - x[i] for i in range(10)] if neg else x)


D_ED = (-121665 * pow(121666, P - 2, P)) % P


def _ed_add(p1, p2):
    x1, y1 = p1; x2, y2 = p2
    t = D_ED * x1 * x2 * y1 * y2 % P
    return ((x1 * y2 + y1 * x2) * pow(1 + t, P - 2, P) % P, (y1 * y2 + x1 * x2) * pow(1 - t, P - 2, P) % P)


def _limbs(x):
    out = []
    for i in range(10):
        w = (26 if i % 2 == 0 else 25)
        out.append(x >> POS[i] & ((1 << w) - 1))
    return out


def test_dbl_host_projective(lib):
    """ge_dbl (negated E' and G', every output coordinate negated: the same
    projective point) against affine big-int doubling from random multiples of
    the base point, projectively scaled by a random Z."""
    rng = random.Random(31)
    by = 4 * pow(5, P - 2, P) % P
    bx2 = (by * by - 1) * pow(D_ED * by * by + 1, P - 2, P) % P
    bx = pow(bx2, (P + 3) // 8, P)
    if (bx * bx - bx2) % P:
        bx = bx * pow(2, (P - 1) // 4, P) % P
    if bx & 1:
        bx = P - bx
    pt = (bx, by)
    for it in range(60):
        pt = _ed_add(pt, (bx, by)) if it % 3 else _ed_add(pt, pt)
        z = rng.randrange(1, P)
        X, Y, Z, T = pt[0] * z % P, pt[1] * z % P, z, pt[0] * pt[1] * z % P
        inp = _limbs(X) + _limbs(Y) + _limbs(Z) + _limbs(T)
        o = (ctypes.c_uint32 * 40)(); lib.t_dbl(o, arr(inp)); o = list(o)
        X3, Y3, Z3, T3 = (val(o[10 * k:10 * k + 10]) % P for k in range(4))
        ex = _ed_add(pt, pt)
        zi = pow(Z3, P - 2, P)
        assert (X3 * zi % P, Y3 * zi % P) == ex
        assert T3 * Z3 % P == X3 * Y3 % P
        assert all(in_R(o[10 * k:10 * k + 10]) for k in range(4))


def test_pipe_recoding(lib):
    """The verify kernels' scalar recoding (fd_scalar_dev.h recode_p_top /
    ybias_p / recode_p_low / recode_p_hi, compiled for the host; ydig_p in
    fd_ed25519_gpu_kern.hip reads the same bits out of LDS): for the wave's
    top-digit position P = clamp(nbits - 3, 124, 252) every scalar x < 2^nbits
    is the sum of its signed digits -- windows 0..nw-3 4-bit in [-8, 8),
    window nw-2 wn bits in [-2^(wn-1), 2^(wn-1)), the top digit in [0, 8] at
    bit P -- so the chain's P doublings and the 9-entry tables (|d| <= 8)
    cover it.  The same digits from a Python restatement."""
    rng = random.Random(77)
    lib.t_recode_p_top.restype = ctypes.c_int

    def model(x, P):
        m = (P + 3) >> 2
        wn = P - 4 * (m - 1)
        nw = m + 1
        y = x + sum(8 << (4 * i) for i in range(m - 1)) + (1 << (4 * (m - 1) + wn - 1))
        assert y < 2**256 and y >> P <= 8                 # nothing above the top digit
        d = [((y >> (4 * i)) & 15) - 8 for i in range(nw - 2)]
        d.append(((y >> (4 * (nw - 2))) & ((1 << wn) - 1)) - (1 << (wn - 1)))
        d.append(y >> P)
        return d, [4 * i for i in range(nw - 1)] + [P], wn

    for nbits in list(range(1, 254)) + [128, 129, 130, 131, 132, 133, 134] * 20:
        P = lib.t_recode_p_top(nbits)
        assert P == min(252, max(124, nbits - 3))
        for x in [(1 << nbits) - 1, 1 << (nbits - 1), rng.randrange(1 << nbits), 0]:
            d, pos, wn = model(x, P)
            assert sum(di << p for di, p in zip(d, pos)) == x
            assert 0 <= d[-1] <= 8
            assert all(-8 <= di < 8 for di in d[:-2]) and -(1 << (wn - 1)) <= d[-2] < (1 << (wn - 1))
            assert pos[-1] == P and pos[-1] - pos[-2] == wn     # the chain's doublings: P in all
            o = (ctypes.c_uint8 * 64)()
            lib.t_recode_p(o, arr([(x >> (32 * j)) & 0xffffffff for j in range(8)]), P)
            assert [o[i] - 8 for i in range(len(d))] == d


def test_is_zero_r(lib):
    """fe_is_zero (one carry pass, then 0 or p) on R-form limbs: equals
    value % p == 0 at the R bounds, for 0 and p in many limb forms and for
    values just past 2^255."""
    rng = random.Random(91)
    lib.t_is_zero.restype = ctypes.c_int
    pl = [2**26 - 19] + [(2**25 - 1) if i & 1 else (2**26 - 1) for i in range(1, 10)]

    def limbs(x):            # a random R-form representation of x (x < 2^255 + small)
        h = []
        for i in range(10):
            w = 25 if i & 1 else 26
            h.append(x & ((1 << w) - 1)); x >>= w
        h[9] += x << 25 if x else 0
        for _ in range(rng.randrange(4)):                  # move carries down within R bounds
            i = rng.randrange(9)
            w = 25 if i & 1 else 26
            if h[i + 1] > 0 and h[i] + (1 << w) <= (R_O if i & 1 else R_E):
                h[i + 1] -= 1; h[i] += 1 << w
        return h
    cases = [[0] * 10, pl, [R_E, R_O] * 5, [x + (1 << 11) if i % 2 == 0 else x for i, x in enumerate(pl)]]
    for _ in range(3000):
        cases.append(limbs(rng.randrange(P)))
        cases.append(limbs(rng.choice([0, P, rng.randrange(2**255, 2**255 + 2**200)])))
        cases.append([rng.randrange(R_E + 1) if i % 2 == 0 else rng.randrange(R_O + 1) for i in range(10)])
    for h in cases:
        assert all(v < 2**31 for v in h)
        assert lib.t_is_zero(arr(h)) == (val(h) % P == 0), h


def test_decode_small_order_flag(lib):
    """ge_decode_small's order <= 8 flag (x == 0 from the decode's own bytes,
    y in {0, p, y0, y1} read off the encoding) equals the affine test on
    the decoded point, for the small-order encodings, y = p + v, random
    encodings and both sign bits, in both decode rules."""
    rng = random.Random(92)
    y0 = 0x05fc536d880238b13933c6d305acdfd5f098eff289f4c345b027b2c28f95e826
    y1 = 0x7a03ac9277fdc74ec6cc392cfa53202a0f67100d760b3cba4fd84d3d706a17c7
    ys = [0, 1, P - 1, P, y0, y1, P - y0, P - y1, 2**255 - 1] + [P + v for v in range(19)]
    ys += [rng.randrange(2**255) for _ in range(400)]
    sm, sma = ctypes.c_int(), ctypes.c_int()
    for y in ys:
        for sign in (0, 1):
            e = y | (sign << 255)
            w = arr([(e >> (32 * j)) & 0xffffffff for j in range(8)])
            for rule in (0, 1):
                ok = lib.t_decode_small(w, rule, ctypes.byref(sm), ctypes.byref(sma))
                if ok:
                    assert sm.value == sma.value, (hex(y), sign, rule)
