#!/usr/bin/env python3
"""make_verify_fixtures.py -- regenerates tests/golden/verify_txns.json
(dev container only; TEST INFRASTRUCTURE).

Inputs: the four transactions of the reference verify-tile test
(src/app/fdctl/run/tiles/test_verify.c:4-109: valid_txn_1sig,
invalid_txn_same_1sig, valid_txn_2sigs, invalid_txn_2sigs), read as hex
data from that file.  For each, the fixture records the payload and the
fd_txn_t the REFERENCE fd_txn_parse produces for it (oracle/_ref,
fdref_txn_parse), so the GPU box can rebuild the tile's frags without the
reference.  The expected per-call results are the FD_TEST assertions of
test_verify.c:144-264, restated in tests/test_verify_stage.py.
"""
import ctypes
import json
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
SRC = "/root/reference/src/app/fdctl/run/tiles/test_verify.c"
NAMES = ["valid_txn_1sig", "invalid_txn_same_1sig", "valid_txn_2sigs", "invalid_txn_2sigs"]


def main():
    text = open(SRC).read()
    ref = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libfdref_avx512.so"))
    ref.fdref_txn_parse.restype = ctypes.c_ulong
    ref.fdref_txn_parse.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_char_p]
    out = {"source": "src/app/fdctl/run/tiles/test_verify.c (hex txns) + reference fd_txn_parse", "txns": {}}
    for name in NAMES:
        m = re.search(r"\b%s\[\]\s*=\s*\{(.*?)\};" % re.escape(name), text, re.S)
        payload = bytes.fromhex("".join(re.findall(r'"([0-9a-fA-F]*)"', m.group(1))))
        buf = ctypes.create_string_buffer(852)
        sz = ref.fdref_txn_parse(payload, len(payload), buf)
        assert sz, name
        out["txns"][name] = {"payload": payload.hex(), "txn_t": buf.raw[:sz].hex()}
    json.dump(out, open(os.path.join(HERE, "verify_txns.json"), "w"), indent=1)
    print({k: len(v["payload"]) // 2 for k, v in out["txns"].items()})


if __name__ == "__main__":
    main()
