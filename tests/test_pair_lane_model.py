"""The pair-lane latency kernel's round, modelled on the CPU (csrc/sha256.hip,
sha256_chain2): two lanes share one message, the E lane keeps (e, f, g, h),
the A lane (a, b, c, d), both run the same instruction stream and three DPP
adds exchange the round's results.  This model executes that stream lane by
lane, with the DPP semantics the kernel relies on (row_shl:4 / row_shr:4
inside rows of 16 lanes, bank masks that enable banks of 4 lanes, disabled
lanes keeping the destination's old value), and compares whole messages with
hashlib (FIPS 180-4; the reference's MessageDigest, StorageNode.java:603-613).
No GPU needed: it pins the algebra (Maj(a, b, c) = Ch(a ^ c, b, c), Z = h + K
+ W one round ahead, the register rotation) and the lane layout."""
import hashlib
import struct

import numpy as np

K = np.array([
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2],
    dtype=np.uint32)
H0 = [0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19]
LANES = np.arange(64)
IS_A = (LANES & 4) != 0            # banks 1 and 3 of every row of 16
E_BANKS, A_BANKS = 0x5, 0xA


def rotr(x, n):
    n = n.astype(np.uint32) if isinstance(n, np.ndarray) else np.uint32(n)
    return (x >> n) | (x << (np.uint32(32) - n))


def bank_enabled(mask):
    return ((mask >> ((LANES % 16) // 4)) & 1).astype(bool)


def dpp_add(dst, src0, src1, ctrl, bank_mask):
    """v_add_u32_dpp dst, src0, src1: src0 permuted inside each row of 16
    lanes; lanes whose source falls outside the row, or whose bank is masked
    off, keep dst."""
    if ctrl == "row_shl:4":      # lane i reads lane i + 4
        src_lane, ok = LANES + 4, (LANES % 16) + 4 < 16
    elif ctrl == "row_shr:4":    # lane i reads lane i - 4
        src_lane, ok = LANES - 4, (LANES % 16) - 4 >= 0
    else:                        # quad_perm:[0,1,2,3]
        src_lane, ok = LANES, np.ones(64, bool)
    write = ok & bank_enabled(bank_mask)
    out = dst.copy()
    out[write] = src0[src_lane[write]] + src1[write]
    return out


def pair_index(lane):
    return ((lane >> 3) << 2) | (lane & 3)


def schedule_kw(block):
    """K[t] + W[t] of one 64-byte block (the helper wave's output)."""
    w = list(struct.unpack(">16I", block))
    for t in range(16, 64):
        s0 = (w[t - 15] >> 7 | w[t - 15] << 25) ^ (w[t - 15] >> 18 | w[t - 15] << 14) ^ (w[t - 15] >> 3)
        s1 = (w[t - 2] >> 17 | w[t - 2] << 15) ^ (w[t - 2] >> 19 | w[t - 2] << 13) ^ (w[t - 2] >> 10)
        w.append((w[t - 16] + s0 + w[t - 7] + s1) & 0xffffffff)
    return (np.array(w, dtype=np.uint64) + K).astype(np.uint32)


def owner_block(st, kw):
    """One block on the owner wave: st[4][64] (per lane: E lanes e..h, A lanes
    a..d), kw[64 rounds][64 lanes] (only the E lanes' values matter)."""
    with np.errstate(over="ignore"):
        s0 = np.where(IS_A, 2, 6).astype(np.uint32)
        s1 = np.where(IS_A, 13, 11).astype(np.uint32)
        s2 = np.where(IS_A, 22, 25).astype(np.uint32)
        m = np.where(IS_A, 0xffffffff, 0).astype(np.uint32)
        x = [v.copy() for v in st]
        z = dpp_add(np.zeros(64, np.uint32), x[3], kw[0], "quad_perm", E_BANKS)
        for t in range(64):
            x0, x1, x2, x3 = x
            s = rotr(x0, s0) ^ rotr(x0, s1) ^ rotr(x0, s2)
            tt = x0 ^ (x2 & m)
            f = (tt & x1) | (~tt & x2)
            y = s + f + z
            x3 = dpp_add(x3, x3, y, "row_shl:4", E_BANKS)          # e' = d + T1
            if t < 63:
                z = dpp_add(z, x2, kw[t + 1], "quad_perm", E_BANKS)  # h of the next round is this round's g
            x3 = dpp_add(x3, y, y, "row_shr:4", A_BANKS)           # a' = T1 + T2
            x = [x3, x0, x1, x2]
        return [st[i] + x[i] for i in range(4)]


def pad(msg):
    n = len(msg)
    msg += b"\x80" + b"\0" * ((55 - n) % 64) + struct.pack(">Q", 8 * n)
    return [msg[i:i + 64] for i in range(0, len(msg), 64)]


def test_lane_layout():
    idx = pair_index(LANES)
    assert sorted(idx.tolist()) == sorted(list(range(32)) * 2)          # every message on exactly two lanes
    assert all(idx[l] == idx[l ^ 4] and IS_A[l] != IS_A[l ^ 4] for l in LANES)  # partner = lane ^ 4, one E + one A
    assert (bank_enabled(E_BANKS) == ~IS_A).all() and (bank_enabled(A_BANKS) == IS_A).all()
    assert ((LANES // 16) == ((LANES ^ 4) // 16)).all()                 # partners share a row of 16


def test_maj_is_ch_of_a_xor_c():
    rng = np.random.default_rng(3)
    a, b, c = (rng.integers(0, 1 << 32, 1000, dtype=np.uint64).astype(np.uint32) for _ in range(3))
    t = a ^ c
    assert (((t & b) | (~t & c)) == ((a & b) ^ (a & c) ^ (b & c))).all()


def test_pair_lane_rounds_match_hashlib():
    """32 messages of ragged lengths (padding boundaries included) through the
    modelled owner wave, block by block; lanes past their own last block keep
    their state, as in the kernel."""
    rng = np.random.default_rng(11)
    lens = [0, 1, 55, 56, 63, 64, 65, 119, 120, 127, 128] + [int(v) for v in rng.integers(0, 400, 21)]
    msgs = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    blocks = [pad(m) for m in msgs]
    idx = pair_index(LANES)
    st = [np.where(IS_A, H0[i], H0[4 + i]).astype(np.uint32) for i in range(4)]
    for k in range(max(len(b) for b in blocks)):
        kw = np.zeros((64, 64), np.uint32)
        act = np.zeros(64, bool)
        for lane in LANES:
            bl = blocks[idx[lane]]
            if k < len(bl):
                kw[:, lane] = schedule_kw(bl[k])
                act[lane] = True
        new = owner_block(st, kw)
        st = [np.where(act, new[i], st[i]) for i in range(4)]
    for p, msg in enumerate(msgs):
        a_lane = next(l for l in LANES if idx[l] == p and IS_A[l])
        e_lane = a_lane ^ 4
        digest = b"".join(struct.pack(">I", int(st[i][a_lane])) for i in range(4)) + \
            b"".join(struct.pack(">I", int(st[i][e_lane])) for i in range(4))
        assert digest == hashlib.sha256(msg).digest(), (p, len(msg))
