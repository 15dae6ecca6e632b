"""Readers for the committed golden fixtures (format: tests/golden/make_golden.py docstring)."""
import os
import struct

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def read_sigs(name):
    """-> list of dict(set, tc_id, code, code_ref, ok, msg, sig, pub)."""
    data = open(os.path.join(GOLDEN, name), "rb").read()
    out, off = [], 0
    while off < len(data):
        set_id, tc_id, ca, cr, ok, _, msg_sz = struct.unpack_from("<IIbbbBI", data, off)
        off += 16
        sig = data[off:off + 64]; pub = data[off + 64:off + 96]; off += 96
        msg = data[off:off + msg_sz]; off += msg_sz
        out.append(dict(set=set_id, tc_id=tc_id, code=ca, code_ref=cr, ok=ok, msg=msg, sig=sig, pub=pub))
    return out


def read_txns(name="txn_batches.bin"):
    """-> list of dict(n, code, code_ref, msg, sigs[list], pubs[list])."""
    data = open(os.path.join(GOLDEN, name), "rb").read()
    out, off = [], 0
    while off < len(data):
        n, msg_sz, ca, cr, _ = struct.unpack_from("<IIbbH", data, off)
        off += 12
        sigs = [data[off + 64 * j:off + 64 * j + 64] for j in range(n)]; off += 64 * n
        pubs = [data[off + 32 * j:off + 32 * j + 32] for j in range(n)]; off += 32 * n
        msg = data[off:off + msg_sz]; off += msg_sz
        out.append(dict(n=n, code=ca, code_ref=cr, msg=msg, sigs=sigs, pubs=pubs))
    return out


def read_sha(name="sha512_kat.bin", dlen=None):
    """[(msg, digest)] of a KAT file (digest 64 B for sha512_kat.bin, 32 B for sha256_kat.bin)."""
    dlen = dlen or (32 if "256" in name else 64)
    data = open(os.path.join(GOLDEN, name), "rb").read()
    out, off = [], 0
    while off < len(data):
        (sz,) = struct.unpack_from("<I", data, off); off += 4
        md = data[off:off + dlen]; off += dlen
        out.append((data[off:off + sz], md)); off += sz
    return out


def read_gossip(name="gossip.bin"):
    """-> (self_pubkey, list of dict(tag, pkt, triples: None (does not decode) or
    list of dict(kind, msg, sig, key, code)))."""
    data = open(os.path.join(GOLDEN, name), "rb").read()
    me, off, out = data[:32], 32, []
    while off < len(data):
        tag, sz, nt = struct.unpack_from("<IIi", data, off); off += 12
        pkt = data[off:off + sz]; off += sz
        trs = None if nt < 0 else []
        for _ in range(max(nt, 0)):
            kind, msz = struct.unpack_from("<II", data, off); off += 8
            msg = data[off:off + msz]; off += msz
            sig = data[off:off + 64]; key = data[off + 64:off + 96]; off += 96
            (code,) = struct.unpack_from("<i", data, off); off += 4
            trs.append(dict(kind=kind, msg=msg, sig=sig, key=key, code=code))
        out.append(dict(tag=tag, pkt=pkt, triples=trs))
    return me, out


def read_shreds(name="shreds.bin"):
    """-> list of dict(tag, result, root, leader, shred) (shreds.bin: make_golden.py gen_shreds)."""
    data = open(os.path.join(GOLDEN, name), "rb").read()
    out, off = [], 0
    while off < len(data):
        tag, sz, r = struct.unpack_from("<IIi", data, off); off += 12
        root = data[off:off + 32]; leader = data[off + 32:off + 64]; off += 64
        out.append(dict(tag=tag, result=r, root=root, leader=leader, shred=data[off:off + sz])); off += sz
    return out
