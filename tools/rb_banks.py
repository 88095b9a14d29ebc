"""LDS bank-conflict model of the fused ResBlock's MFMA operand reads (csrc/tvq_resblock.hip).

ds_read_b32: two 32-lane groups, bank = (byte address / 4) mod 32; each extra distinct
address on a bank within a group costs one cycle (MI355X_MICROARCH.md §LDS).  The model
counts, per image (block), the extra cycles of the conv B-operand reads (halo-plane gathers,
forward and the flipped data gradient) and of the weight-gradient A (dY plane) and B (input
window) reads, for a layout (row stride WP, plane stride PS) and an operand order:
  'base': the round-3 kernels (WP = W + 2, PS == 2 mod 32, k = 4 s + kq, positions p0 + kq);
  'pair': the reduction index of lanes kq and kq ^ 1 paired at an address distance of 16
          (mod 32), weight-gradient positions w and w + 16 (W >= 32) as the pair.
Usage: python tools/rb_banks.py  (prints the per-kernel extra cycles for C/W = 8/64, 16/32,
32/16 under both; the chosen WP / PS search is `best_layout`).
"""
import itertools


def geom(C, W, RB_NW=8):
    P = 3 * W
    MT = P // 16
    NR = (C + 15) // 16
    NCH0 = min(C // 4, RB_NW // NR)
    NCH = min(NCH0, 4)
    CPC = C // NCH
    CMS = RB_NW // (NR * NCH)
    CNF = (MT + CMS - 1) // CMS
    K = 9 * C
    KC = K + 1
    KT = (KC + 15) // 16
    WPS0 = 1 if C >= 32 else (8 if (C == 8 and W >= 32) else 4)
    WPS = min(WPS0, RB_NW)
    WKG = RB_NW // WPS
    WNF = (KT + WKG - 1) // WKG
    WSTEPS = (P // 4) // WPS
    return dict(P=P, MT=MT, NR=NR, NCH=NCH, CPC=CPC, CMS=CMS, CNF=CNF, K=K, KC=KC, KT=KT,
                WPS=WPS, WKG=WKG, WNF=WNF, WSTEPS=WSTEPS)


def conflicts(addrs):
    """extra cycles of one ds_read_b32 given 64 lane addresses (None = lane reads nothing)"""
    extra = 0
    for g in (range(0, 32), range(32, 64)):
        banks = {}
        for l in g:
            a = addrs[l]
            if a is None:
                continue
            banks.setdefault(a % 32, set()).add(a)
        extra += max((len(s) for s in banks.values()), default=1) - 1
    return extra


def tap_off(t, WP):
    return (t // 3) * WP + t % 3


def pairing(offs):
    """order the chunk's reductions (with plane offsets offs[r]) into quads (kq 0..3) so
    that kq 0/1 and 2/3 are 16 apart mod 32 where possible (greedy matching)"""
    n = len(offs)
    left = list(range(n))
    pairs = []
    while left:
        r = left.pop(0)
        mate = None
        for q in left:
            if (offs[q] - offs[r]) % 32 == 16:
                mate = q
                break
        if mate is None:  # least-bad partner: distance farthest from 0 mod 32
            mate = max(left, key=lambda q: min((offs[q] - offs[r]) % 32, (offs[r] - offs[q]) % 32))
        left.remove(mate)
        pairs.append((r, mate))
    quads = []
    for i in range(0, len(pairs), 2):
        quads.append(pairs[i] + pairs[i + 1])
    return quads


def model(C, W, mode, WP=None, PS=None):
    g = geom(C, W)
    if mode == "base":
        WP = W + 2
        HW = 5 * WP
        PS = HW + ((2 - HW % 32) + 32) % 32
    pos = lambda p: (p // W) * WP + p % W  # noqa: E731
    out = {}
    for flip in (False, True):
        total = 0
        for wid in range(8):
            m = wid % g["CMS"]
            combo = wid // g["CMS"]
            ch = combo % g["NCH"]
            nsteps = 9 * g["CPC"] // 4
            if mode == "base":
                order = [tuple(4 * s + kq for kq in range(4)) for s in range(nsteps)]
            else:
                offs = []
                for r in range(9 * g["CPC"]):
                    c, t = r // 9, r % 9
                    offs.append(c * PS + tap_off(8 - t if flip else t, WP))
                order = pairing(offs)
            for f in range(g["CNF"]):
                mt = m + g["CMS"] * f
                mt = mt if mt < g["MT"] else m
                for s in range(nsteps):
                    addrs = []
                    for l in range(64):
                        j, kq = l & 15, l >> 4
                        r = order[s][kq]
                        c, t = r // 9, r % 9
                        if flip:
                            t = 8 - t
                        a = ch * g["CPC"] * PS + c * PS + tap_off(t, WP) + pos(mt * 16 + j)
                        addrs.append(a)
                    total += conflicts(addrs)
        out["conv_bwd" if flip else "conv_fwd"] = total
    # weight gradient
    tA = tB = 0
    for wid in range(8):
        kg = wid % g["WKG"]
        pc = wid // g["WKG"]
        for s in range(g["WSTEPS"]):
            S = pc * g["WSTEPS"] + s  # global step (4 positions)
            if mode == "base" or W < 32:
                ps = [4 * S + kq for kq in range(4)]
            else:
                blk, i = S // 8, S % 8
                ps = [32 * blk + (kq & 1) * 16 + 2 * i + (kq >> 1) for kq in range(4)]
            for nr in range(g["NR"]):
                addrs = []
                for l in range(64):
                    j, kq = l & 15, l >> 4
                    n = nr * 16 + j
                    addrs.append(n * PS + pos(ps[kq]) if n < C else 10 ** 6 + pos(ps[kq]))
                tA += conflicts(addrs)
            for f in range(g["WNF"]):
                kt = kg + g["WKG"] * f
                addrs = []
                for l in range(64):
                    j, kq = l & 15, l >> 4
                    kc = kt * 16 + j
                    if kc < g["K"]:
                        c, t = kc // 9, kc % 9
                        base = c * PS + tap_off(t, WP)
                    else:
                        base = 2 * 10 ** 6 if kc == g["K"] else 3 * 10 ** 6
                    addrs.append(base + pos(ps[kq]))
                tB += conflicts(addrs)
    out["wgrad_A"] = tA
    out["wgrad_B"] = tB
    out["WP"], out["PS"] = WP, PS
    return out


def lin_layout(W):
    """the round-4 layout: row stride WP == 3 and plane stride PS == 9 (mod 32), so the
    window cell of reduction index r = c*9 + t sits at bank r (mod 32)"""
    WP = W + 2 + ((3 - (W + 2) % 32) + 32) % 32
    PS = 5 * WP + ((9 - (5 * WP) % 32) + 32) % 32
    return WP, PS


def lin_order(N):
    """closed-form quads: r and r + 16 share a lane pair within each 32-block of the
    chunk's N reductions; the tail (N mod 32) in consecutive quads"""
    nb = N // 32
    out = []
    for s in range(N // 4):
        if s < 8 * nb:
            b, i = s // 8, s % 8
            out.append(tuple(32 * b + 2 * i + (kq & 1) * 16 + (kq >> 1) for kq in range(4)))
        else:
            out.append(tuple(32 * nb + 4 * (s - 8 * nb) + kq for kq in range(4)))
    return out


def model_lin(C, W, k1res):
    """'lin' layout with exact LDS bases: G plane at 0, S plane at C*PS, ones plane K1 at
    residue k1res (mod 32), zeros plane K0 = K1 + PS"""
    g = geom(C, W)
    WP, PS = lin_layout(W)
    pos = lambda p: (p // W) * WP + p % W  # noqa: E731
    Sb = C * PS
    K1 = 10 ** 6 * 32 + k1res
    K0 = K1 + PS
    out = {}
    N = 9 * g["CPC"]
    order = lin_order(N)
    for flip in (False, True):
        total = 0
        for wid in range(8):
            m = wid % g["CMS"]
            ch = (wid // g["CMS"]) % g["NCH"]
            for f in range(g["CNF"]):
                mt = m + g["CMS"] * f
                mt = mt if mt < g["MT"] else m
                for s in range(N // 4):
                    addrs = []
                    for l in range(64):
                        j, kq = l & 15, l >> 4
                        r = order[s][kq]
                        c, t = r // 9, r % 9  # flip: the panel holds the reversed tap
                        addrs.append(ch * g["CPC"] * PS + c * PS + tap_off(t, WP) + pos(mt * 16 + j))
                    total += conflicts(addrs)
        out["conv_bwd" if flip else "conv_fwd"] = total
    tA = tB = 0
    for wid in range(8):
        kg, pc = wid % g["WKG"], wid // g["WKG"]
        for s in range(g["WSTEPS"]):
            S = pc * g["WSTEPS"] + s
            if W >= 32:
                blk, i = S // 8, S % 8
                ps = [32 * blk + (kq & 1) * 16 + 2 * i + (kq >> 1) for kq in range(4)]
            else:
                ps = [4 * S + kq for kq in range(4)]
            for nr in range(g["NR"]):
                addrs = []
                for l in range(64):
                    j, kq = l & 15, l >> 4
                    n = nr * 16 + j
                    addrs.append((n * PS if n < C else K0) + WP + 1 + pos(ps[kq]))
                tA += conflicts(addrs)
            for f in range(g["WNF"]):
                kt = kg + g["WKG"] * f
                addrs = []
                for l in range(64):
                    j, kq = l & 15, l >> 4
                    kc = kt * 16 + j
                    if kc < g["K"]:
                        c, t = kc // 9, kc % 9
                        base = Sb + c * PS + tap_off(t, WP)
                    else:
                        base = K1 if kc == g["K"] else K0
                    addrs.append(base + pos(ps[kq]))
                tB += conflicts(addrs)
    out["wgrad_A"], out["wgrad_B"] = tA, tB
    out["WP"], out["PS"] = WP, PS
    return out


def best_layout(C, W):
    best = None
    for WP in range(W + 2, W + 2 + 32):
        for PS in range(5 * WP, 5 * WP + 32):
            r = model(C, W, "pair", WP, PS)
            cost = r["conv_fwd"] + r["conv_bwd"] + r["wgrad_A"] + r["wgrad_B"]
            key = (cost, PS)
            if best is None or key < best[0]:
                best = (key, r)
    return best[1]


if __name__ == "__main__":
    import sys
    for C, W in ((8, 64), (16, 32), (32, 16), (8, 32), (16, 64), (8, 16), (16, 16), (32, 32)):
        b = model(C, W, "base")
        tot = lambda r: 2 * r["conv_fwd"] + 2 * (r["conv_bwd"] + r["wgrad_A"] + r["wgrad_B"])  # noqa
        best = min(((tot(model_lin(C, W, k)), k) for k in range(32)))
        print(C, W, "base", tot(b), b)
        print(C, W, "lin ", best[0], "k1res", best[1], model_lin(C, W, best[1]))
        if "--search" in sys.argv:
            print(C, W, "best", best_layout(C, W))
