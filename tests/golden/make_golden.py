#!/usr/bin/env python3
"""make_golden.py -- regenerates the committed golden fixtures (dev container only).

TEST INFRASTRUCTURE.  Needs /root/reference (the reference sources) and the
reference libraries built by `make -C oracle ref`.  The fixtures it writes are
plain data (inputs + expected codes); nothing from the reference is copied.

Where expected codes come from
  * code_avx512: the reference fd_ed25519_verify compiled with FD_HAS_AVX512
    (oracle/_ref/libfdref_avx512.so) -- the backend the reference's
    config/machine/native.mk picks on an AVX-512-IFMA host and the CPU path
    bench.py times.  This is THE golden code.
  * code_ref: the same sources compiled for the portable `ref` backend.
    Recorded for information (the two differ on pubkey-decode failures,
    SURVEY.md §8(a) A4/A5).
  * ok: the accept/reject the reference's own test files assert
    (test_ed25519_wycheproof.c / test_ed25519_cctv.c `.ok`, the two
    malleability .bin files); -1 where the reference tests say nothing.

Files written (tests/golden/):
  vectors_ref.bin   Wycheproof (set 1), CCTV (set 2), malleability fail/pass (sets 4/5)
  synthetic.bin     config-1 valid sigs (set 10), adversarial classes (sets 20..39),
                    variable-length messages 0..1232 B (set 11)
  txn_batches.bin   multi-signature single-message batches (A2 precedence)
  sha512_kat.bin    SHA-512 known answers (fd_sha512_test_vector.c + CAVP ShortMsg/LongMsg)
  cctv_batches.bin  the reference's own batch scenario, test_cctv_batch
                    (src/ballet/ed25519/test_ed25519.c:1041-1082): 16 fresh valid
                    signatures over CCTV message #7, then each CCTV vector with that
                    message at slot 1 of 2- and 4-signature batches (txn format; the
                    reference's `ok` re-asserted on the batch codes)
  fuzz_seeds.bin    the 4 corpus/fuzz_ed25519_sigverify seeds through the harness of
                    src/ballet/ed25519/fuzz_ed25519_sigverify.c:30-49 (seed = prv[32] || msg:
                    public_from_private, sign, verify must be SUCCESS), as sig records
                    (set 50), reference codes recorded

  gossip.bin        gossip packets -- the reference's own gossip fixtures
                    (src/flamenco/types/fixtures/gossip_*.bin: a pull request, pull
                    responses carrying contact-info v1/v2, node-instance, snapshot-hash
                    and version values, a push of a vote) plus ping / pong / prune
                    packets signed by the reference signer and malformed variants --
                    with the (msg, sig, key, code) triples the REFERENCE gossip code
                    forms for each (oracle/ref_gossip.c: the reference decoder,
                    encoder and fd_ed25519_verify)

  shreds.bin        shreds -- the 480 of the reference's demo capture
                    (src/disco/shred/fixtures/demo-shreds.pcap, leader key
                    demo-shreds.key) plus corrupted variants -- with the result of
                    the REFERENCE FEC resolver's first-shred check (oracle/ref_shred.c:
                    the reference fd_shred_parse, bmtree, SHA-256, fd_ed25519_verify)

`python3 make_golden.py cctv_batches.bin fuzz_seeds.bin` rewrites only the named files.

Record format (ed25519 files), little endian:
  u32 set, u32 tc_id, i8 code_avx512, i8 code_ref, i8 ok, u8 0, u32 msg_sz,
  u8 sig[64], u8 pub[32], u8 msg[msg_sz]
txn_batches.bin record:
  u32 n, u32 msg_sz, i8 code_avx512, i8 code_ref, u16 0, u8 sigs[64n], u8 pubs[32n], u8 msg[msg_sz]
sha512_kat.bin record:
  u32 msg_sz, u8 digest[64], u8 msg[msg_sz]
sha256_kat.bin record (fd_sha256_test_vector.c + CAVP SHA256{Short,Long}Msg.rsp, every 4th):
  u32 msg_sz, u8 digest[32], u8 msg[msg_sz]
shreds.bin record:
  u32 tag, u32 sz, i32 result (verify code, or -101..-106 as oracle/ref_shred.c), u8 root[32],
  u8 leader[32], u8 shred[sz]
gossip.bin: u8 self[32], then per packet:
  u32 tag, u32 pkt_sz, i32 ntriples (-1: the packet does not decode), u8 pkt[pkt_sz],
  ntriples x { u32 kind, u32 msg_sz, u8 msg[msg_sz], u8 sig[64], u8 key[32], i32 code }
"""
import ctypes
import os
import struct
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_SRC = os.environ.get("FD_REF_SRC", "/root/reference/src")

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
# y coordinates of the order-8 points, as listed in src/ballet/ed25519/fd_curve25519.h:86-93
Y0 = int.from_bytes(bytes.fromhex("26e8958fc2b227b045c3f489f2ef98f0d5dfac05d3c63339b13802886d53fc05"), "little")
Y1 = int.from_bytes(bytes.fromhex("c7176a703d4dd84fba3c0b760d10670f2a2053fa2c39ccc64ec7fd7792ac037a"), "little")


def load_libs():
    libs = {}
    for b in ("avx512", "ref"):
        lib = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libfdref_%s.so" % b))
        lib.fdref_verify.restype = ctypes.c_int
        lib.fdref_verify.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p]
        lib.fdref_verify_batch_single_msg.restype = ctypes.c_int
        lib.fdref_verify_batch_single_msg.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p,
                                                      ctypes.c_char_p, ctypes.c_ulong]
        lib.fdref_sign.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p]
        lib.fdref_public_from_private.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        lib.fdref_shred_check.restype = ctypes.c_int
        lib.fdref_shred_check.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p]
        lib.fdref_gossip_triples.restype = ctypes.c_long
        lib.fdref_gossip_triples.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p, ctypes.c_char_p,
                                             ctypes.c_ulong]
        assert lib.fdref_backend_avx512() == (1 if b == "avx512" else 0)
        libs[b] = lib
    return libs


LIBS = None


def verify(msg, sig, pub):
    return tuple(LIBS[b].fdref_verify(msg, len(msg), sig, pub) for b in ("avx512", "ref"))


def verify_batch(msg, sigs, pubs, n):
    return tuple(LIBS[b].fdref_verify_batch_single_msg(msg, len(msg), sigs, pubs, n) for b in ("avx512", "ref"))


def keypair(rng):
    priv = rng.bytes(32)
    pub = ctypes.create_string_buffer(32)
    LIBS["avx512"].fdref_public_from_private(pub, priv)
    return priv, pub.raw


def sign(msg, pub, priv):
    sig = ctypes.create_string_buffer(64)
    LIBS["avx512"].fdref_sign(sig, msg, len(msg), pub, priv)
    return sig.raw


def rec(set_id, tc_id, codes, ok, msg, sig, pub):
    assert len(sig) == 64 and len(pub) == 32
    return struct.pack("<IIbbbBI", set_id, tc_id, codes[0], codes[1], ok, 0, len(msg)) + sig + pub + msg


def enc(y, sign_bit):
    return (y | (sign_bit << 255)).to_bytes(32, "little")


def extract_reference_vectors():
    exe = "/tmp/fdgpu_extract_vectors"
    out = "/tmp/fdgpu_vectors.bin"
    cmd = ["gcc", "-std=c17", "-O1", "-w", "-I" + REF_SRC, "-DFD_HAS_HOSTED=1", "-D_XOPEN_SOURCE=700",
           "-DFD_HAS_INT128=1", "-DFD_HAS_DOUBLE=1", "-DFD_HAS_X86=1", "-DFD_HAS_SSE=1", "-DFD_HAS_AVX=1",
           "-o", exe, os.path.join(HERE, "extract_vectors.c")]
    subprocess.check_call(cmd)
    subprocess.check_call([exe, out])
    data = open(out, "rb").read()
    vecs, off = [], 0
    while off < len(data):
        set_id, tc_id, ok, msg_sz = struct.unpack_from("<IIiI", data, off)
        off += 16
        sig = data[off:off + 64]; pub = data[off + 64:off + 96]; off += 96
        msg = data[off:off + msg_sz]; off += msg_sz
        vecs.append((set_id, tc_id, ok, msg, sig, pub))
    return vecs


def gen_vectors_ref(vecs):
    out = []
    for set_id, tc_id, ok, msg, sig, pub in vecs:
        if set_id in (1, 2):
            out.append(rec(set_id, tc_id, verify(msg, sig, pub), ok, msg, sig, pub))
    # malleability records: 96-byte {sig, pub}, msg "Zcash"
    # (src/ballet/ed25519/test_ed25519_signature_malleability.c:4-15,21)
    for set_id, fname, ok in ((4, "should_fail", 0), (5, "should_pass", 1)):
        path = os.path.join(REF_SRC, "ballet/ed25519/test_ed25519_signature_malleability_%s.bin" % fname)
        raw = open(path, "rb").read()
        assert len(raw) % 96 == 0
        for i in range(len(raw) // 96):
            sig = raw[96 * i:96 * i + 64]; pub = raw[96 * i + 64:96 * i + 96]
            out.append(rec(set_id, i, verify(b"Zcash", sig, pub), ok, b"Zcash", sig, pub))
    return out


def gen_synthetic():
    rng = np.random.default_rng(1234)
    out = []
    # set 10: config 1 -- 1024 distinct keys, 200-byte random messages, all valid
    keys = [keypair(rng) for _ in range(1024)]
    for i, (priv, pub) in enumerate(keys):
        msg = rng.bytes(200)
        sig = sign(msg, pub, priv)
        c = verify(msg, sig, pub)
        assert c == (0, 0)
        out.append(rec(10, i, c, 1, msg, sig, pub))
    # set 11: config 3 shape -- message length uniform in 0..1232 (MTU), all valid
    for i in range(256):
        priv, pub = keys[i]
        msg = rng.bytes(int(rng.integers(0, 1233)))
        sig = sign(msg, pub, priv)
        c = verify(msg, sig, pub)
        assert c == (0, 0)
        out.append(rec(11, i, c, 1, msg, sig, pub))
    # explicit SHA block-boundary lengths: 64+msg+17 crosses 128*k
    for j, m in enumerate([0, 1, 46, 47, 48, 63, 64, 110, 111, 112, 127, 128, 175, 176, 239, 240, 1231, 1232]):
        priv, pub = keys[j]
        msg = rng.bytes(m)
        sig = sign(msg, pub, priv)
        out.append(rec(12, j, verify(msg, sig, pub), 1, msg, sig, pub))

    def base(i, n=200):
        priv, pub = keys[i % len(keys)]
        msg = rng.bytes(n)
        return msg, sign(msg, pub, priv), pub, priv

    tc = 0

    def add(set_id, msg, sig, pub, ok=-1):
        nonlocal tc
        out.append(rec(set_id, tc, verify(msg, sig, pub), ok, msg, sig, pub))
        tc += 1

    for i in range(64):   # set 20: 1-bit flip in the message -> ERR_MSG
        msg, sig, pub, _ = base(i)
        b = bytearray(msg); b[i % len(b)] ^= 1 << (i % 8)
        add(20, bytes(b), sig, pub, 0)
    for i in range(64):   # set 21: 1-bit flip in S low bytes
        msg, sig, pub, _ = base(i)
        s = bytearray(sig); s[32 + (i % 16)] ^= 1 << (i % 8)
        add(21, msg, bytes(s), pub, 0)
    for i in range(32):   # set 22: S >= L via the high byte -> ERR_SIG
        msg, sig, pub, _ = base(i)
        s = bytearray(sig); s[63] |= (0x10, 0x20, 0x40, 0x80)[i % 4]
        add(22, msg, bytes(s), pub, 0)
    for i, S in enumerate([L, L - 1, L + 1, 2**256 - 1, 2**253, 0, 1]):   # set 23: scalar boundaries
        msg, sig, pub, _ = base(i)
        add(23, msg, sig[:32] + S.to_bytes(32, "little"), pub, -1)
    for i in range(128):  # set 24: random pubkey bytes (about half do not decode)
        msg, sig, _, _ = base(i)
        add(24, msg, sig, rng.bytes(32), 0)
    for i in range(128):  # set 25: random R bytes
        msg, sig, pub, _ = base(i)
        add(25, msg, rng.bytes(32) + sig[32:], pub, 0)
    # set 26/27: x=0 encodings with sign bit 1 (y = 1, y = p-1) as A / as R
    for i, y in enumerate([1, P - 1, P + 1]):
        for sgn in (0, 1):
            msg, sig, pub, _ = base(i)
            add(26, msg, sig, enc(y, sgn), 0)
            add(27, msg, enc(y, sgn) + sig[32:], pub, 0)
    # set 28/29: non-canonical y = p + v, v in [0, 18], both signs, as A / as R
    for v in range(19):
        for sgn in (0, 1):
            msg, sig, pub, _ = base(v)
            add(28, msg, sig, enc(P + v, sgn), 0)
            add(29, msg, enc(P + v, sgn) + sig[32:], pub, 0)
    # set 30/31: the small-order y's (0, 1, p-1, y0, y1) and their +p aliases, both signs
    for y in (0, 1, P - 1, Y0, Y1, P, P + 1):
        for sgn in (0, 1):
            if y >= 2**255:
                continue
            msg, sig, pub, _ = base(y & 0xff)
            add(30, msg, sig, enc(y, sgn), 0)
            add(31, msg, enc(y, sgn) + sig[32:], pub, 0)
    # set 32: small-order A with a signature made to verify against it is impossible
    # without the private key; instead mixed-order A = A_valid + T (torsion): sign
    # with the honest key, publish the torsioned key -> equation fails (cofactorless)
    # Covered by CCTV; here random full-order A with R swapped between two valid sigs.
    for i in range(32):
        msg, sig, pub, _ = base(i)
        msg2, sig2, pub2, _ = base(i + 1)
        add(32, msg, sig2[:32] + sig[32:], pub, 0)
    # set 33: empty and single-byte messages, valid
    for i, n in enumerate([0, 1, 2, 3]):
        msg, sig, pub, _ = base(i, n)
        add(33, msg, sig, pub, 1)
    return out


def gen_txn_batches():
    rng = np.random.default_rng(4321)
    keys = [keypair(rng) for _ in range(64)]
    out = []

    def one(n, corrupt):
        msg = rng.bytes(int(rng.integers(0, 600)))
        sigs, pubs = [], []
        for j in range(max(n, 1)):
            priv, pub = keys[int(rng.integers(0, len(keys)))]
            sig = sign(msg, pub, priv)
            kind = corrupt.get(j)
            if kind == "msg":       # wrong signature (other message) -> -3 in phase 2
                sig = sign(msg + b"x", pub, priv)
            elif kind == "S":       # S >= L -> -1 in phase 1
                sig = sig[:63] + bytes([sig[63] | 0xf0])
            elif kind == "A_small":  # small-order A -> -2 in phase 1
                pub = enc(0, 0)
            elif kind == "A_bad":   # undecodable A (y=2: u=3,v=4d+1 non-square) -> -1 avx512 / -2 ref
                pub = enc(2, 0)
            elif kind == "R_small":  # small-order R -> -1
                sig = enc(1, 0) + sig[32:]
            sigs.append(sig); pubs.append(pub)
        sigs_b = b"".join(sigs[:n] if n else sigs[:0]); pubs_b = b"".join(pubs[:n] if n else pubs[:0])
        pad_s = sigs_b if n else bytes(64); pad_p = pubs_b if n else bytes(32)
        codes = verify_batch(msg, pad_s, pad_p, n)
        out.append(struct.pack("<IIbbH", n, len(msg), codes[0], codes[1], 0) + sigs_b + pubs_b + msg)

    kinds = ["msg", "S", "A_small", "A_bad", "R_small"]
    for n in range(1, 13):
        one(n, {})
    # every ordered pair of failure kinds at two positions (probes the two-phase precedence)
    for a in kinds:
        for b in kinds:
            for n in (2, 3, 5):
                one(n, {0: a, 1: b})
                one(n, {n - 1: a, 0: b})
    for _ in range(64):
        n = int(rng.integers(1, 13))
        corrupt = {int(rng.integers(0, n)): kinds[int(rng.integers(0, len(kinds)))] for _ in range(int(rng.integers(0, 3)))}
        one(n, corrupt)
    one(16, {})
    one(16, {15: "msg"})
    one(17, {})            # n > 16 -> -1 before any work (fd_ed25519_user.c:238-240)
    one(0, {})             # n == 0 -> -1
    return out


def gen_cctv_batches(vecs):
    """test_cctv_batch (test_ed25519.c:1041-1082) as fixtures: the reference
    draws the 16 keys from fd_rng(seed 0); any 16 fresh keys exercise the same
    scenario, so ours come from a fixed numpy seed and the reference signer."""
    cctv = [v for v in vecs if v[0] == 2]
    msg = cctv[7][3]
    rng = np.random.default_rng(1041)
    sigs, pubs = [], []
    for _ in range(16):
        priv, pub = keypair(rng)
        sigs.append(sign(msg, pub, priv)); pubs.append(pub)
    assert verify_batch(msg, b"".join(sigs), b"".join(pubs), 16) == (0, 0)     # :1057
    out = []
    for set_id, tc_id, ok, m, sig, pub in cctv:
        if m != msg:
            continue
        s2 = list(sigs); p2 = list(pubs)
        s2[1] = sig; p2[1] = pub                                                   # :1069-1070
        for n in (2, 4):                                                           # :1072, :1076
            sb = b"".join(s2[:n]); pb = b"".join(p2[:n])
            codes = verify_batch(msg, sb, pb, n)
            if ok in (0, 1):
                assert (codes[0] == 0) == bool(ok), (tc_id, n, codes, ok)
            out.append(struct.pack("<IIbbH", n, len(msg), codes[0], codes[1], tc_id & 0xffff) + sb + pb + msg)
    return out


def gen_fuzz_seeds():
    """corpus/fuzz_ed25519_sigverify/* through LLVMFuzzerTestOneInput
    (fuzz_ed25519_sigverify.c:30-49): input = prv[32] || msg."""
    d = os.path.join(os.path.dirname(REF_SRC), "corpus", "fuzz_ed25519_sigverify")
    out = []
    for i, name in enumerate(sorted(os.listdir(d))):
        data = open(os.path.join(d, name), "rb").read()
        if len(data) < 32:                      # :31 returns early
            continue
        priv, msg = data[:32], data[32:]
        pub = ctypes.create_string_buffer(32)
        LIBS["avx512"].fdref_public_from_private(pub, priv)
        sig = sign(msg, pub.raw, priv)
        codes = verify(msg, sig, pub.raw)
        assert codes == (0, 0), (name, codes)  # :46-47
        out.append(rec(50, i, codes, 1, msg, sig, pub.raw))
    return out


GOSSIP_SELF = bytes(range(100, 132))


def gossip_triples(pkt, me=GOSSIP_SELF):
    """The reference gossip code's triples for one packet (oracle/ref_gossip.c)."""
    buf = ctypes.create_string_buffer(1 << 20)
    n = LIBS["avx512"].fdref_gossip_triples(pkt, len(pkt), me, buf, len(buf))
    assert n >= -1, n
    if n < 0:
        return None
    out, at = [], 0
    raw = buf.raw
    for _ in range(n):
        kind, msz = struct.unpack_from("<II", raw, at); at += 8
        msg = raw[at:at + msz]; at += msz
        sig = raw[at:at + 64]; at += 64
        key = raw[at:at + 32]; at += 32
        code, = struct.unpack_from("<i", raw, at); at += 4
        out.append((kind, msg, sig, key, code))
    return out


def gen_gossip():
    """Gossip packets and the reference's triples (fd_gossip.c:474-484, 735-762,
    830-900, 1002-1030 via oracle/ref_gossip.c)."""
    pkts = []
    fx = os.path.join(REF_SRC, "flamenco/types/fixtures")
    for i, name in enumerate(sorted(f for f in os.listdir(fx) if f.startswith("gossip_") and f.endswith(".bin"))):
        pkts.append((100 + i, open(os.path.join(fx, name), "rb").read()))
    rng = np.random.default_rng(1589)
    keys = [keypair(rng) for _ in range(4)]
    # ping / pong: {u32 kind, from, token, signature}
    for kind in (4, 5):
        for t in range(6):
            priv, pub = keys[t % 4]
            token = rng.bytes(32)
            sig = sign(token, pub, priv)
            p = struct.pack("<I", kind) + pub + token + sig
            if t == 1:
                p = p[:100] + bytes([p[100] ^ 4]) + p[101:]          # signature bit flip
            elif t == 2:
                p = p[:40] + bytes([p[40] ^ 1]) + p[41:]             # token bit flip
            elif t == 3:
                p = p + b"\0"                                       # a byte over
            elif t == 4:
                p = p[:-1]                                           # a byte short
            elif t == 5:
                p = struct.pack("<I", kind) + rng.bytes(32) + token + sig   # a key that may not decode
            pkts.append((kind * 10 + t, p))

    def prune(priv, pub, inner, prunes, dest, wall, nfield=None, tail=b""):
        n = len(prunes) if nfield is None else nfield
        body = lambda sig: (struct.pack("<I", 3) + pub + inner + struct.pack("<Q", n) + b"".join(prunes) + sig +
                            dest + struct.pack("<Q", wall) + tail)
        tr = gossip_triples(body(bytes(64)), me=dest)
        if not tr:
            return body(rng.bytes(64))
        return body(sign(tr[0][1], pub, priv))
    for t in range(12):
        priv, pub = keys[t % 4]
        pr = [rng.bytes(32) for _ in range((0, 1, 3, 20)[t % 4])]
        wall = int(rng.integers(0, 2**62))
        inner = pub if t % 3 else keys[(t + 1) % 4][1]
        if t == 5:
            p = prune(priv, pub, inner, pr, rng.bytes(32), wall)               # not for this node
        elif t == 6:
            p = bytearray(prune(priv, pub, inner, pr, GOSSIP_SELF, wall)); p[-50] ^= 0x10; p = bytes(p)
        elif t == 7:
            p = prune(priv, pub, inner, pr, GOSSIP_SELF, wall, nfield=len(pr) + 1)   # count past the data
        elif t == 8:
            p = prune(priv, pub, inner, pr, GOSSIP_SELF, wall, nfield=1 << 63)
        elif t == 9:
            p = prune(priv, pub, inner, pr, GOSSIP_SELF, wall, tail=b"\1\2")       # bytes over
        else:
            p = prune(priv, pub, inner, pr, GOSSIP_SELF, wall)
        pkts.append((60 + t, p))
    # pull responses / pushes over every CRDS variant, values signed over the
    # REFERENCE encoder's bytes (so only a walk that re-encodes exactly as
    # fd_crds_data_encode does verifies them): one per signer, one of this
    # node's (filtered), one with a flipped signature bit, one unsigned
    sys.path.insert(0, os.path.dirname(HERE))
    import crds_gen
    for disc in range(12):
        for t in range(2):
            priv, pub = keys[(disc + t) % 4]
            sender = pub if disc == 11 else rng.bytes(32)   # contact-info v2: the message's key signs
            body = None
            while body is None or gossip_triples(pkt) is None:        # votes: the packet's tail must parse as a txn
              body = []
              for i, (d, key) in enumerate([(disc, pub), (disc, GOSSIP_SELF), (disc, pub), ((disc + 5) % 12, None)]):
                dat = crds_gen.data(rng, d, rng.bytes(32) if key is None else key)
                one = struct.pack("<I", 2) + sender + struct.pack("<Q", 1) + bytes(64) + dat
                tr = gossip_triples(one, me=None)
                sig = sign(tr[0][1], pub, priv) if (i < 3 and tr) else rng.bytes(64)
                if i == 2:
                    sig = sig[:5] + bytes([sig[5] ^ 0x20]) + sig[6:]
                body.append(sig + dat)
              pkt = struct.pack("<I", 1 + t) + sender + struct.pack("<Q", len(body)) + b"".join(body)
            pkts.append((200 + 2 * disc + t, pkt))
    pkts.append((90, struct.pack("<I", 7) + rng.bytes(128)))                 # unknown kind
    pkts.append((91, b"\4\0\0"))                                             # short
    out = [GOSSIP_SELF]
    for tag, p in pkts:
        tr = gossip_triples(p)
        out.append(struct.pack("<IIi", tag, len(p), -1 if tr is None else len(tr)) + p)
        for kind, msg, sig, key, code in tr or []:
            out.append(struct.pack("<II", kind, len(msg)) + msg + sig + key + struct.pack("<i", code))
    return out


def shred_check(sh, leader):
    """the reference FEC resolver's first-shred check (oracle/ref_shred.c)"""
    root = ctypes.create_string_buffer(32)
    r = LIBS["avx512"].fdref_shred_check(sh, len(sh), leader, root)
    return r, (root.raw if r > -100 else bytes(32))


def gen_shreds():
    """The reference's demo shred capture (fd_fec_resolver tests' fixtures)
    and corrupted variants, with the reference resolver's check."""
    d = os.path.join(REF_SRC, "disco/shred/fixtures")
    leader = open(os.path.join(d, "demo-shreds.key"), "rb").read()[32:]
    cap = open(os.path.join(d, "demo-shreds.pcap"), "rb").read()
    shreds, off = [], 24
    while off < len(cap):
        incl, = struct.unpack_from("<I", cap, off + 8); off += 16
        shreds.append(cap[off + 42:off + incl]); off += incl      # Ethernet + IPv4 + UDP headers
    rng = np.random.default_rng(399)
    other = keypair(rng)[1]
    recs = [(i, sh, leader) for i, sh in enumerate(shreds)]

    def put16(b, o, v):
        b[o:o + 2] = struct.pack("<H", v & 0xffff)

    def put32(b, o, v):
        b[o:o + 4] = struct.pack("<I", v & 0xffffffff)
    data = [sh for sh in shreds if sh[0x40] & 0xf0 == 0x80]
    code = [sh for sh in shreds if sh[0x40] & 0xf0 == 0x40]
    for t in range(48):
        base = bytearray((data if t % 2 else code)[int(rng.integers(0, 240))])
        k = t // 2
        if k == 0:   base[100 + int(rng.integers(0, 900))] ^= 1                      # protected byte
        elif k == 1: base[len(base) - 1 - int(rng.integers(0, 20 * (base[0x40] & 0xf)))] ^= 0x40   # proof byte
        elif k == 2: base[0:64] = bytes(64)                                          # zero signature
        elif k == 3: base[5] ^= 0x80                                                 # signature bit
        elif k == 4: base[32:64] = (L + int(rng.integers(0, 1000))).to_bytes(32, "little")   # S >= l
        elif k == 5: base = base[:-1]                                                # a byte short
        elif k == 6: base[0x40] = (base[0x40] & 0xf0) | ((base[0x40] + 1) & 0xf)    # proof length + 1
        elif k == 7: base[0x40] = (base[0x40] & 0xf0) | ((base[0x40] - 1) & 0xf)    # proof length - 1
        elif k == 8: base[0x40] = (base[0x40] & 0xf0)                                # no proof
        elif k == 9: base[0x40] = 0x5a if t % 2 == 0 else 0x20 | (base[0x40] & 0xf)  # legacy code / bad type
        elif k == 10:
            if t % 2: put32(base, 0x49, struct.unpack_from("<I", base, 0x4f)[0] - 1)    # idx below its set
            else: put16(base, 0x53, 0)                                                # data count 0
        elif k == 11:
            if t % 2: put32(base, 0x49, struct.unpack_from("<I", base, 0x4f)[0] + 66)  # index 66: deeper than the proof
            else: put16(base, 0x53, 68)                                               # data count 68
        elif k == 12:
            if t % 2: put16(base, 0x56, 0x50)                                         # data size below the header
            else: put16(base, 0x55, 0)                                                # code count 0
        elif k == 13:
            if t % 2: base = base + bytes(25)                                         # extra bytes after a data shred
            else: put16(base, 0x57, 67)                                               # coding index 67
        elif k == 14: base = base + bytes(3)                                          # bytes over
        elif k == 15: recs.append((1000 + t, bytes(base), other)); continue           # another leader
        elif k == 16: base[0x41] ^= 1                                                  # slot (unprotected? no: in the leaf)
        else: base[64 + int(rng.integers(0, 0x18))] ^= 0x10                          # header bytes
        recs.append((1000 + t, bytes(base), leader))
    out = []
    for tag, sh, ld in recs:
        r, root = shred_check(sh, ld)
        out.append(struct.pack("<IIi", tag, len(sh), r) + root + ld + sh)
    return out


def gen_sha512(vecs):
    out = []
    for set_id, tc_id, ok, msg, sig, pub in vecs:
        if set_id == 3:
            out.append(struct.pack("<I", len(msg)) + sig + msg)
    # NIST CAVP (src/ballet/sha512/cavp/SHA512{Short,Long}Msg.rsp), every 4th record
    for fname in ("SHA512ShortMsg.rsp", "SHA512LongMsg.rsp"):
        path = os.path.join(REF_SRC, "ballet/sha512/cavp", fname)
        ln = None; msg = None; k = 0
        for line in open(path):
            line = line.strip()
            if line.startswith("Len ="):
                ln = int(line.split("=")[1])
            elif line.startswith("Msg ="):
                msg = bytes.fromhex(line.split("=")[1].strip())[: ln // 8]
            elif line.startswith("MD ="):
                md = bytes.fromhex(line.split("=")[1].strip())
                if k % 4 == 0:
                    out.append(struct.pack("<I", len(msg)) + md + msg)
                k += 1
    return out


def gen_sha256(vecs):
    out = []
    for set_id, tc_id, ok, msg, sig, pub in vecs:
        if set_id == 4:
            out.append(struct.pack("<I", len(msg)) + sig[:32] + msg)
    # NIST CAVP (src/ballet/sha256/cavp/SHA256{Short,Long}Msg.rsp), every 4th record
    for fname in ("SHA256ShortMsg.rsp", "SHA256LongMsg.rsp"):
        path = os.path.join(REF_SRC, "ballet/sha256/cavp", fname)
        ln = None; msg = None; k = 0
        for line in open(path):
            line = line.strip()
            if line.startswith("Len ="):
                ln = int(line.split("=")[1])
            elif line.startswith("Msg ="):
                msg = bytes.fromhex(line.split("=")[1].strip())[: ln // 8]
            elif line.startswith("MD ="):
                md = bytes.fromhex(line.split("=")[1].strip())
                if k % 4 == 0:
                    out.append(struct.pack("<I", len(msg)) + md + msg)
                k += 1
    return out


def main():
    global LIBS
    LIBS = load_libs()
    vecs = extract_reference_vectors()
    gens = {"vectors_ref.bin": lambda: gen_vectors_ref(vecs), "synthetic.bin": gen_synthetic,
            "txn_batches.bin": gen_txn_batches, "sha512_kat.bin": lambda: gen_sha512(vecs),
            "sha256_kat.bin": lambda: gen_sha256(vecs),
            "cctv_batches.bin": lambda: gen_cctv_batches(vecs), "fuzz_seeds.bin": gen_fuzz_seeds,
            "gossip.bin": gen_gossip, "shreds.bin": gen_shreds}
    only = sys.argv[1:] or list(gens)
    for name in only:
        recs = gens[name]()
        with open(os.path.join(HERE, name), "wb") as f:
            f.write(b"".join(recs))
        print(name, len(recs), "records", file=sys.stderr)


if __name__ == "__main__":
    main()
