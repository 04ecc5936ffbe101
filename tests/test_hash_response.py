"""The reply half of the storeFragments exchange (host functions of the C
ABI, no GPU needed): dfs_store_hash_responses_build against the oracle's
buildHashResponse (StorageNode.java:644-655, HashMap iteration order
included) and dfs_store_hash_responses_check against the oracle's
parseResponseHashes + the sender's comparison (:657-701, :248-257), on good
replies, tampered / missing / reordered / duplicated entries, odd spacing and
the inputs where the Java parser throws."""
import ctypes
import hashlib
import random

import numpy as np

import oracle as O
from dfs_amd import _lib as L

OK, MISMATCH, WIRE = 0, L.DFS_E_FRAG_MISMATCH, L.DFS_E_WIRE


def _build(file_ids, idx, digs, status=None):
    n = len(file_ids)
    ids = np.frombuffer("".join(file_ids).encode(), np.uint8).copy() if n else np.zeros(1, np.uint8)
    fi = np.array(idx, np.uint32).reshape(-1)
    dg = np.frombuffer(b"".join(a + b for a, b in digs), np.uint8).copy() if n else np.zeros(1, np.uint8)
    st = np.array(status, np.int32) if status is not None else None
    off = np.zeros(n + 1, np.uint64)
    cap = int(L.lib().dfs_store_hash_response_cap()) * max(n, 1)
    out = np.zeros(cap, np.uint8)
    rc = L.lib().dfs_store_hash_responses_build(ids.ctypes.data, fi.ctypes.data, dg.ctypes.data,
                                                st.ctypes.data if st is not None else None, n, out.ctypes.data, cap,
                                                off.ctypes.data)
    assert rc == 0
    return [out[int(off[i]):int(off[i + 1])].tobytes().decode() for i in range(n)]


def _check(replies, idx, digs):
    n = len(replies)
    blob = "".join(replies).encode()
    spans = (L.dfs_span * max(n, 1))()
    o = 0
    for i, r in enumerate(replies):
        spans[i].off, spans[i].len = o, len(r.encode())
        o += len(r.encode())
    buf = np.frombuffer(blob or b"\0", np.uint8).copy()
    fi = np.array(idx, np.uint32).reshape(-1)
    dg = np.frombuffer(b"".join(a + b for a, b in digs), np.uint8).copy()
    st = np.full(n, 99, np.int32)
    rc = L.lib().dfs_store_hash_responses_check(buf.ctypes.data, spans, n, fi.ctypes.data, dg.ctypes.data, st.ctypes.data)
    return rc, st.tolist()


def _expected_status(reply, pair, digs):
    """The reference: parseResponseHashes, then f.hash.equals(remote.get(f.index)) for both fragments."""
    try:
        m = O.py_parse_response_hashes(reply)
    except O.JavaException:
        return WIRE
    for k, d in zip(pair, digs):
        if m.get(k) != d.hex():
            return MISMATCH
    return OK


def test_build_matches_the_references_reply():
    rng = random.Random(5)
    ids, idx, digs = [], [], []
    for case in range(200):
        fid = hashlib.sha256(b"f%d" % case).hexdigest()
        n = rng.choice([2, 5, 8, 10, 17, 40])
        a = rng.randrange(n)
        b = (a + 1) % n if rng.random() < 0.8 else rng.randrange(n)  # also a == b and far pairs (bucket order)
        ids.append(fid)
        idx.append((a, b))
        digs.append((hashlib.sha256(b"a%d" % case).digest(), hashlib.sha256(b"b%d" % case).digest()))
    got = _build(ids, idx, digs)
    for i in range(len(ids)):
        want = O.py_build_hash_response(ids[i], [(idx[i][0], digs[i][0].hex()), (idx[i][1], digs[i][1].hex())])
        assert got[i] == want, i
        assert len(got[i]) <= L.lib().dfs_store_hash_response_cap()
    # a body that failed on the receiver gets no reply; the others are unchanged
    st = [0, L.DFS_E_DECODE, 0, L.DFS_E_WIRE] + [0] * (len(ids) - 4)
    part = _build(ids, idx, digs, st)
    assert part[1] == "" and part[3] == "" and part[0] == got[0] and part[2] == got[2] and part[4:] == got[4:]
    assert _build([], [], []) == []


def test_check_matches_the_references_parser_and_comparison():
    rng = random.Random(9)
    fid = hashlib.sha256(b"x").hexdigest()
    pair = (4, 0)
    d = (hashlib.sha256(b"frag4").digest(), hashlib.sha256(b"frag0").digest())
    good = O.py_build_hash_response(fid, [(4, d[0].hex()), (0, d[1].hex())])
    e4 = '{"index":"4","hash":"%s"}' % d[0].hex()
    e0 = '{"index":"0","hash":"%s"}' % d[1].hex()
    head = '{"fileId":"%s","received":[' % fid
    replies = [
        good,
        head + e4 + "," + e0 + "]}",                        # the other order
        "  \n" + good + "\t ",                             # trimmed
        good.replace('"hash":"', '"hash": "'),              # spaces after the colon
        head + e0 + "]}",                                  # fragment 4 missing
        good.replace(d[0].hex(), hashlib.sha256(b"other").hexdigest()),  # wrong hash
        good.replace(d[1].hex()[:8], d[1].hex()[:8].upper()) if d[1].hex()[:8].upper() != d[1].hex()[:8] else good[:-1],
        head + e4 + "," + e0 + "," + '{"index":"0","hash":"%s"}' % ("0" * 64) + "]}",  # a later entry replaces index 0
        head + '{"index":"x","hash":"%s"}' % d[0].hex() + "," + e0 + "]}",  # parseInt throws
        head + '{"index":"99999999999","hash":"ab"}' + "]}",               # out of int range
        '{"fileId":"%s"}' % fid,                            # no "received"
        '{"received":]',                                    # ']' before '[' + 1: substring throws? (no '[')
        ']"received"[',                                     # '[' after, ']' none after it
        '"received"[]',                                     # empty array
        '"received"][',                                     # ']' found from index of '[' on: none -> empty map
        "",                                                 # no reply at all
        head + e4 + ",{" + e0[1:] + "]}",                   # "},{" split still finds both
        head + '{"hash":"%s","index":"4"}' % d[0].hex() + "," + e0 + "]}",  # fields swapped
        head + '{"index":"+4","hash":"%s"}' % d[0].hex() + "," + e0 + "]}",  # parseInt accepts a sign
    ]
    for _ in range(60):  # random damage to a good reply
        s = list(good)
        for _ in range(rng.randrange(1, 4)):
            p = rng.randrange(len(s))
            s[p] = rng.choice('{}[]",:x0 ')
        replies.append("".join(s))
    idx = [pair] * len(replies)
    digs = [d] * len(replies)
    rc, st = _check(replies, idx, digs)
    want = [_expected_status(r, pair, d) for r in replies]
    assert st == want, [(i, replies[i], st[i], want[i]) for i in range(len(replies)) if st[i] != want[i]][:3]
    assert want[0] == OK and want[1] == OK and want[4] == MISMATCH and want[5] == MISMATCH and want[8] == WIRE
    assert rc == next(s for s in st if s != OK)
    # what the build half writes, the check half accepts, for every pair of a 10-fragment upload
    ids, idx2, digs2 = [], [], []
    for a in range(10):
        ids.append(fid)
        idx2.append((a, (a + 1) % 10))
        digs2.append((hashlib.sha256(b"p%d" % a).digest(), hashlib.sha256(b"q%d" % a).digest()))
    rc, st = _check(_build(ids, idx2, digs2), idx2, digs2)
    assert rc == OK and st == [OK] * 10
