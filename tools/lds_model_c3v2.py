"""LDS bank model for the conv3 backward v2 layouts (MI355X_MICROARCH.md §LDS lane groups / bank rules).
Prints the LDS cycles per wave-instruction (ideal = the group count) for every access pattern."""
import itertools

RB128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
         list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
RB128 += [[l + 32 for l in g] for g in RB128]
G2x32 = [list(range(32)), list(range(32, 64))]
W128 = [list(range(8 * i, 8 * i + 8)) for i in range(8)]


def cycles(addrs, nbytes, groups, nbanks):
    """addrs: lane -> byte address; returns LDS cycles (max distinct addresses per bank, summed per group)."""
    tot = 0
    for g in groups:
        banks = {}
        for l in g:
            a = addrs[l]
            for d in range(nbytes // 4):
                b = (a // 4 + d) % nbanks
                banks.setdefault(b, set()).add(a // 4 + d)
        tot += max(len(v) for v in banks.values())
    return tot


def tr16(addrs):  # ds_read_b64_tr_b16: 8 B per lane, 2 x 32 groups, 64 banks
    return cycles(addrs, 8, G2x32, 64)


# ---------------------------------------------------------------- dgrad P: [64 pos][128 co] bf16
def p_off(pos, co, mode):
    if mode == "pad136":
        return pos * 272 + co * 2
    ch = co // 8  # 16-B chunk (16 per row)
    if mode == "xor":
        return pos * 256 + 16 * (ch ^ (pos & 15)) + (co % 8) * 2
    if mode == "xor2":
        return pos * 256 + 16 * (ch ^ ((pos * 3) & 15)) + (co % 8) * 2


for mode in ("pad136", "xor", "xor2"):
    worst_r = 0
    for mt in range(4):
        for ks in range(4):
            ad = [p_off(16 * mt + (l & 15), ks * 32 + (l >> 4) * 8, mode) for l in range(64)]
            worst_r = max(worst_r, cycles(ad, 16, RB128, 64))
    # expansion writes: thread t -> window w = t >> 4, 8-channel group c8 = t & 15, row i
    worst_w = 0
    for wave in range(4):
        for i in range(4):
            ad = []
            for l in range(64):
                t = wave * 64 + l
                w, c8 = t >> 4, t & 15
                pos = (2 * (w >> 2) + (i >> 1)) * 8 + 2 * (w & 3) + (i & 1)
                ad.append(p_off(pos, c8 * 8, mode))
            worst_w = max(worst_w, cycles(ad, 16, W128, 32))
    print(f"P {mode:7s}: B-frag read {worst_r} (ideal 4), expansion write {worst_w} (ideal 8)")


# ---------------------------------------------------------------- dgrad DA: [100 q][64 ci] fp32
def key(y, x):
    return (x + 8 * (y & 1)) & 15


def da_off(y, x, ci, mode):
    c = ci // 4
    if mode == "pad68":
        return (y * 10 + x) * 272 + ci * 4
    return (y * 10 + x) * 256 + 16 * (c ^ key(y, x)) + (ci % 4) * 4


for mode in ("pad68", "xor"):
    worst_rmw_r = worst_rmw_w = 0
    for wave, half, m, ty, tx in itertools.product(range(4), range(2), range(2), range(3), range(3)):
        ad = []
        for l in range(64):
            p = l & 15
            py, px = 2 * (2 * half + m) + (p >> 3), p & 7
            ad.append(da_off(py + ty, px + tx, 16 * wave + (l >> 4) * 4, mode))
        worst_rmw_r = max(worst_rmw_r, cycles(ad, 16, RB128, 64))
        worst_rmw_w = max(worst_rmw_w, cycles(ad, 16, W128, 32))
    # pool2 reads: item (y, cq): lane l of wave w -> item w*48 + l (cq = item & 15, y = item >> 4)
    worst_p = 0
    for wave in range(4):
        for x in range(10):
            ad = []
            for l in range(64):
                it = min(wave * 48 + l, 175)
                y, cq = min(it >> 4, 9), it & 15
                ad.append(da_off(y, x, cq * 4, mode))
            worst_p = max(worst_p, cycles(ad, 16, RB128, 64))
    print(f"DA {mode:6s}: col2im read {worst_rmw_r} (4) write {worst_rmw_w} (8), pool2 read {worst_p} (4)")


# ---------------------------------------------------------------- wgrad D: [64 rows][64 co] bf16, tr16 A reads
def d_off(r, co, rs):
    return r * rs * 2 + co * 2


best = None
for rs in range(64, 96, 4):
    worst = 0
    for ks, mi in itertools.product(range(2), range(4)):
        ad = []
        for l in range(64):
            g16, grp = l & 15, l >> 4
            q, p = g16 >> 2, g16 & 3
            kb = ks * 32 + grp * 8
            ad.append(d_off(kb + q, mi * 16 + 4 * p, rs))
        worst = max(worst, tr16(ad))
    # expansion writes (M-split: 64 co = 8 groups of 8 -> thread t: window t >> 3, c8 = t & 7, 2 threads' rows...)
    worst_w = 0
    for wave in range(4):
        for i in range(4):
            ad = []
            for l in range(64):
                t = wave * 64 + l
                w, c8 = (t >> 3) & 15, t & 7
                ad.append(d_off(4 * w + i, c8 * 8, rs))
            worst_w = max(worst_w, cycles(ad, 16, W128, 32))
    print(f"D rs={rs}: A tr16 read {worst} (2), expansion write {worst_w} (8)")


# ---------------------------------------------------------------- wgrad X: a2 [100 pos][64 ci] bf16, tr16 B reads
def win_pos(r, pw=10):
    w, i = r >> 2, r & 3
    return (2 * (w >> 2) + (i >> 1)) * pw + 2 * (w & 3) + (i & 1)


for rs in range(64, 100, 4):
    worst = 0
    for ks, j, wave in itertools.product(range(2), range(9), range(4)):
        n0 = (9 * wave + j) * 16
        tap, c0 = n0 >> 6, n0 & 63
        shift = (tap // 3) * 10 + tap % 3
        ad = []
        for l in range(64):
            g16, grp = l & 15, l >> 4
            q, p = g16 >> 2, g16 & 3
            kb = ks * 32 + grp * 8
            ad.append((win_pos(kb + q) + shift) * rs * 2 + (c0 + 4 * p) * 2)
        worst = max(worst, tr16(ad))
    # register-staged writes: thread t, k-th chunk c = t + 256 k -> row c >> 3, col (c & 7) * 8
    worst_w = 0
    for k, wave in itertools.product(range(4), range(4)):
        ad = []
        for l in range(64):
            c = min(wave * 64 + l + 256 * k, 799)
            ad.append((c >> 3) * rs * 2 + (c & 7) * 16)
        worst_w = max(worst_w, cycles(ad, 16, W128, 32))
    print(f"X rs={rs}: B tr16 read {worst} (2), staging write {worst_w} (8)")
