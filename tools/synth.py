"""synth.py -- synthetic workload generation for bench.py and the verify-stage
benchmark (NOT part of the product, NOT the oracle):

  * RFC 8032 Ed25519 key generation and signing, hashing with hashlib and
    scalar arithmetic with Python integers, the fixed-base multiplications
    [a]B / [r]B batched in tools/bin/libsynth_sign.so (tools/synth_sign.c,
    host threads);
  * Solana legacy / v0 transactions (wire format of src/ballet/txn/fd_txn.h)
    with n signers, and their parsed fd_txn_t bytes built directly from the
    construction (field layout fd_txn.h:169-288; tests/test_synth.py checks
    them byte for byte against the reference fd_txn_parse);
  * tango frags laid out like fd_tpu_reasm's append_descriptor
    (src/disco/quic/fd_tpu_reasm.c:175-221):
    [payload][pad to 2][fd_txn_t][u16 payload_sz], one per 64-byte-aligned
    chunk like a dcache.
"""
import ctypes
import hashlib
import os
import struct

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
L = 2 ** 252 + 27742317777372353535851937790883648493
FD_TXN_VLEGACY = 0xFF
FD_TXN_V0 = 0x00
FRAG_DTYPE = np.dtype([("off", "<u4"), ("sz", "<u4")])

_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "bin", "libsynth_sign.so")
        if not os.path.exists(path):
            raise RuntimeError("tools/bin/libsynth_sign.so not built (make -C tools)")
        _LIB = ctypes.CDLL(path)
        _LIB.synth_scalarmult_base.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p, ctypes.c_int]
    return _LIB


def scalarmult_base(scalars, threads=16):
    """encode([s]B) for a list of ints (0 <= s < 2^256)."""
    n = len(scalars)
    if not n:
        return []
    buf = b"".join(int(s).to_bytes(32, "little") for s in scalars)
    out = ctypes.create_string_buffer(32 * n)
    _lib().synth_scalarmult_base(buf, n, out, min(threads, max(1, n)))
    raw = out.raw
    return [raw[32 * i:32 * i + 32] for i in range(n)]


def _expand(seed):
    h = hashlib.sha512(seed).digest()
    a = int.from_bytes(h[:32], "little")
    a &= (1 << 254) - 8
    a |= 1 << 254
    return a, h[32:]


def keypairs(seeds, threads=16):
    """[(seed, pub)] for 32-byte seeds (RFC 8032 5.1.5)."""
    ex = [_expand(s) for s in seeds]
    pubs = scalarmult_base([a for a, _ in ex], threads)
    return list(zip(seeds, pubs))


def sign_many(items, threads=16):
    """items: [(seed, pub, msg)] -> [sig] (RFC 8032 5.1.6)."""
    ex = [_expand(s) for s, _, _ in items]
    rs = [int.from_bytes(hashlib.sha512(pre + m).digest(), "little") % L for (_, pre), (_, _, m) in zip(ex, items)]
    Rs = scalarmult_base(rs, threads)
    sigs = []
    for (a, _), r, R, (_, pub, m) in zip(ex, rs, Rs, items):
        k = int.from_bytes(hashlib.sha512(R + pub + m).digest(), "little") % L
        sigs.append(R + ((r + k * a) % L).to_bytes(32, "little"))
    return sigs


def cu16(v):
    """compact-u16 (fd_txn_parse.c READ_CHECKED_COMPACT_U16)."""
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def build_message(rng, signer_pubs, n_extra=2, n_instr=1, data_sz=32, version=FD_TXN_VLEGACY, ro_signed=0,
                  ro_unsigned=1, n_luts=0):
    """Serialize a message; returns (message bytes, layout dict with offsets
    relative to the message start, for the fd_txn_t)."""
    n_sig = len(signer_pubs)
    keys = list(signer_pubs) + [rng.bytes(32) for _ in range(n_extra)]
    n_keys = len(keys)
    m = bytearray()
    if version != FD_TXN_VLEGACY:
        m.append(0x80 | version)
    m += bytes([n_sig, ro_signed, ro_unsigned])
    m += cu16(n_keys)
    acct_off = len(m)
    for k in keys:
        m += k
    rbh_off = len(m)
    m += rng.bytes(32)
    m += cu16(n_instr)
    instrs = []
    for _ in range(n_instr):
        prog = int(rng.integers(1, n_keys))
        accts = [int(x) for x in rng.integers(0, n_keys, size=int(rng.integers(0, 4)))]
        data = rng.bytes(data_sz)
        m.append(prog)
        m += cu16(len(accts))
        a_off = len(m)
        m += bytes(accts)
        m += cu16(len(data))
        d_off = len(m)
        m += data
        instrs.append((prog, len(accts), len(data), a_off, d_off))
    luts = []
    if version != FD_TXN_VLEGACY:
        m += cu16(n_luts)
        for _ in range(n_luts):
            addr_off = len(m)
            m += rng.bytes(32)
            w = [int(x) for x in rng.integers(0, 256, size=1)]
            r = [int(x) for x in rng.integers(0, 256, size=1)]
            m += cu16(len(w))
            w_off = len(m)
            m += bytes(w)
            m += cu16(len(r))
            r_off = len(m)
            m += bytes(r)
            luts.append((addr_off, len(w), len(r), w_off, r_off))
    lay = dict(version=version, n_sig=n_sig, ro_signed=ro_signed, ro_unsigned=ro_unsigned, n_keys=n_keys,
               acct_off=acct_off, rbh_off=rbh_off, instrs=instrs, luts=luts)
    return bytes(m), lay


def txn_t_bytes(lay, message_off):
    """The fd_txn_t the reference parser produces for this construction
    (fd_txn.h:169-288: 20-byte header, 10-byte fd_txn_instr_t entries,
    8-byte fd_txn_acct_addr_lut_t entries), offsets relative to the payload."""
    mo = message_off
    adtl_w = sum(l[1] for l in lay["luts"])
    adtl = sum(l[1] + l[2] for l in lay["luts"])
    b = struct.pack("<BBHHBBHHHBBBBH", lay["version"], lay["n_sig"], 1, mo, lay["ro_signed"], lay["ro_unsigned"],
                    lay["n_keys"], mo + lay["acct_off"], mo + lay["rbh_off"], len(lay["luts"]), adtl_w, adtl, 0,
                    len(lay["instrs"]))
    for prog, ac, ds, ao, do in lay["instrs"]:
        b += struct.pack("<BBHHHH", prog, 0, ac, ds, mo + ao, mo + do)
    for addr_off, wc, rc, wo, ro in lay["luts"]:
        b += struct.pack("<HBBHH", mo + addr_off, wc, rc, mo + wo, mo + ro)
    return b


def build_txns(rng, n_txn, sig_cnts, threads=16, version=FD_TXN_VLEGACY, data_sz=32):
    """n_txn signed transactions with sig_cnts[i] signers each (fresh keys).
    Returns [(payload bytes, fd_txn_t bytes)]."""
    seeds = [[rng.bytes(32) for _ in range(sig_cnts[i])] for i in range(n_txn)]
    flat = [s for ss in seeds for s in ss]
    pubs = [p for _, p in keypairs(flat, threads)]
    msgs, lays, k = [], [], 0
    for i in range(n_txn):
        mp = pubs[k:k + sig_cnts[i]]
        k += sig_cnts[i]
        m, lay = build_message(rng, mp, version=version, data_sz=data_sz,
                               n_luts=(1 if version != FD_TXN_VLEGACY else 0))
        msgs.append(m)
        lays.append(lay)
    items = []
    k = 0
    for i in range(n_txn):
        for j in range(sig_cnts[i]):
            items.append((flat[k + j], pubs[k + j], msgs[i]))
        k += sig_cnts[i]
    sigs = sign_many(items, threads)
    out, k = [], 0
    for i in range(n_txn):
        n = sig_cnts[i]
        payload = cu16(n) + b"".join(sigs[k:k + n]) + msgs[i]
        k += n
        out.append((payload, txn_t_bytes(lays[i], 1 + 64 * n)))
    return out


def pack_frags(txns, chunk=64, extra=0):
    """[(payload, txn_t)] -> (arena uint8, frags FRAG_DTYPE): frag i =
    [payload][pad][fd_txn_t][u16 payload_sz] at a chunk-aligned offset."""
    offs, sizes, blobs = [], [], []
    off = 0
    for payload, txn_t in txns:
        pad = (-len(payload)) % 2
        blob = payload + b"\0" * pad + txn_t + struct.pack("<H", len(payload))
        offs.append(off)
        sizes.append(len(blob))
        blobs.append(blob)
        off += (len(blob) + chunk - 1) // chunk * chunk
    arena = np.zeros(off + extra + 64, np.uint8)
    for o, b in zip(offs, blobs):
        arena[o:o + len(b)] = np.frombuffer(b, np.uint8)
    frags = np.zeros(len(txns), FRAG_DTYPE)
    frags["off"] = offs
    frags["sz"] = sizes
    return arena, frags
