"""Random gossip pull-response / push packets (test data only).

Every CRDS variant of the reference's crds_data (src/flamenco/types/fd_types.json
gossip_* / crds_data), with the encodings the reference decoder accepts but
its encoder does not write back as received: option tags other than 0 / 1,
non-minimal serde varints, the varint-u16 fields of gossip_version_v3 and
gossip_socket_entry (decoded compact-u16, encoded fixed u16), legacy and v0
vote transactions.  Used by tests/golden/make_golden.py (signed fixtures)
and tests/test_gossip.py (a differential fuzz against the reference's own
decoder + encoder, oracle/ref_gossip.c)."""
import struct

import numpy as np


def cu16(v):
    """compact-u16, minimal (the only form fd_bincode_compact_u16_decode takes)"""
    if v < 0x80:
        return bytes([v])
    if v < 0x4000:
        return bytes([(v & 0x7f) | 0x80, v >> 7])
    return bytes([(v & 0x7f) | 0x80, ((v >> 7) & 0x7f) | 0x80, v >> 14])


def varint(v, pad=0):
    """serde varint of v, with pad extra zero groups (non-minimal)"""
    out = bytearray()
    while True:
        if v < 0x80:
            out.append(v)
            break
        out.append((v & 0x7f) | 0x80)
        v >>= 7
    if pad:
        out[-1] |= 0x80
        out += b"\x80" * (pad - 1) + b"\x00"
    return bytes(out)


def u64(v):
    return struct.pack("<Q", v)


def _opt(rng):
    return int(rng.choice([0, 1, 1, 2, 0x80, 0xff]))


def txn(rng, v0=None):
    """a legal transaction as fd_txn_parse_core takes it (legacy or v0)"""
    v0 = bool(rng.integers(0, 2)) if v0 is None else v0
    nsig = int(rng.integers(1, 3))
    ro_u = int(rng.integers(0, 3))
    acct = nsig + ro_u + int(rng.integers(1, 4))
    b = bytes([nsig]) + rng.bytes(64 * nsig)
    b += (bytes([0x80]) if v0 else b"") + bytes([nsig, int(rng.integers(0, nsig)), ro_u])
    b += cu16(acct) + rng.bytes(32 * acct) + rng.bytes(32)
    tables = []
    if v0:
        for _ in range(int(rng.integers(0, 3))):
            w, r = int(rng.integers(0, 3)), int(rng.integers(0, 3))
            if w + r == 0:
                w = 1
            tables.append((w, r))
    adtl = sum(w + r for w, r in tables)
    ninstr = int(rng.integers(0, 4))
    b += cu16(ninstr)
    for _ in range(ninstr):
        k = int(rng.integers(0, 4))
        dl = int(rng.choice([0, 3, 200]))
        b += bytes([int(rng.integers(1, acct))]) + cu16(k) + bytes(int(x) for x in rng.integers(0, acct + adtl, k))
        b += cu16(dl) + rng.bytes(dl)
    if v0:
        b += cu16(len(tables))
        for w, r in tables:
            b += rng.bytes(32) + cu16(w) + rng.bytes(w) + cu16(r) + rng.bytes(r)
    return b


def ip(rng):
    return struct.pack("<I", 0) + rng.bytes(4) if rng.integers(0, 3) else struct.pack("<I", 1) + rng.bytes(16)


def sock(rng):
    return ip(rng) + rng.bytes(2)


def slot_hash(rng):
    return rng.bytes(40)


def vec(rng, el, n=None):
    n = int(rng.integers(0, 4)) if n is None else n
    return u64(n) + b"".join(el(rng) for _ in range(n))


def bytes_vec(rng, n=None):
    n = int(rng.choice([0, 1, 17, 90])) if n is None else n
    return u64(n) + rng.bytes(n)


def _slots(rng):
    if rng.integers(0, 2):
        return struct.pack("<I", 0) + rng.bytes(16) + bytes_vec(rng)
    o = _opt(rng)
    return struct.pack("<I", 1) + rng.bytes(16) + bytes([o]) + (bytes_vec(rng) if o else b"") + rng.bytes(8)


def _v3_u16(rng):
    return cu16(int(rng.choice([0, 5, 127, 128, 300, 16383, 16384, 65535])))


def data(rng, disc, key):
    """crds_data bytes of variant disc whose own key is `key` (32 bytes)"""
    d = struct.pack("<I", disc)
    if disc == 0:
        return d + key + b"".join(sock(rng) for _ in range(10)) + rng.bytes(10)
    if disc == 1:
        return d + rng.bytes(1) + key + txn(rng) + rng.bytes(8)
    if disc == 2:
        return d + rng.bytes(1) + key + rng.bytes(16) + vec(rng, lambda r: r.bytes(8)) + rng.bytes(16)
    if disc in (3, 4):
        return d + key + vec(rng, slot_hash) + rng.bytes(8)
    if disc == 5:
        return d + rng.bytes(1) + key + vec(rng, _slots) + rng.bytes(8)
    if disc in (6, 7):
        o = _opt(rng)
        return d + key + rng.bytes(14) + bytes([o]) + (rng.bytes(4) if o else b"") + (rng.bytes(4) if disc == 7 else b"")
    if disc == 8:
        return d + key + rng.bytes(24)
    if disc == 9:
        return d + rng.bytes(2) + key + rng.bytes(23) + bytes_vec(rng)
    if disc == 10:
        return d + key + slot_hash(rng) + vec(rng, slot_hash) + rng.bytes(8)
    if disc == 11:
        wc = int(rng.integers(0, 2**63))
        pad = int(rng.choice([0, 0, 1, 3, 12]))        # 12: past 64 bits, the decoder's shifts wrap
        b = d + key + varint(wc, pad) + rng.bytes(10)
        b += _v3_u16(rng) + _v3_u16(rng) + _v3_u16(rng) + rng.bytes(8) + _v3_u16(rng)
        na = int(rng.integers(0, 3))
        b += cu16(na) + b"".join(ip(rng) for _ in range(na))
        ns = int(rng.integers(0, 4))
        b += cu16(ns) + b"".join(rng.bytes(2) + _v3_u16(rng) for _ in range(ns))
        ne = int(rng.integers(0, 3))
        return b + cu16(ne) + rng.bytes(4 * ne)
    raise ValueError(disc)


def packet(rng, kind, me, sender, values):
    """{u32 kind (1 pull response / 2 push), sender, u64 n, n x (sig, data)};
    values: list of (disc, key) -- key None: random, "me": this node's"""
    body = []
    for disc, key in values:
        k = me if key == "me" else (rng.bytes(32) if key is None else key)
        body.append(rng.bytes(64) + data(rng, disc, k))
    return struct.pack("<I", kind) + sender + u64(len(body)) + b"".join(body)


def random_packet(rng, me):
    kind = int(rng.integers(1, 3))
    vals = [(int(rng.integers(0, 12)), "me" if rng.integers(0, 8) == 0 else None)
            for _ in range(int(rng.integers(1, 5)))]
    return packet(rng, kind, me, me if rng.integers(0, 6) == 0 else rng.bytes(32), vals)


def mutate(rng, p):
    """flip / insert / delete / truncate a few bytes"""
    p = bytearray(p)
    for _ in range(int(rng.integers(1, 4))):
        op = int(rng.integers(0, 5))
        i = int(rng.integers(0, max(len(p), 1)))
        if op == 0 and p:
            p[i % len(p)] ^= 1 << int(rng.integers(0, 8))
        elif op == 1 and p:
            p[i % len(p)] = int(rng.choice([0, 1, 2, 0x7f, 0x80, 0xff]))
        elif op == 2:
            p[i:i] = rng.bytes(int(rng.integers(1, 4)))
        elif op == 3 and p:
            del p[i:i + int(rng.integers(1, 4))]
        elif p:
            del p[i:]
    return bytes(p)
