# CPU emulation of apg_maze.hpp's precomputed-stream DFS (k_maze_stream's 5-bit outputs, the 32-output window,
# its refill in the memory phase, the permutation read off the window, stalls, the generator past the stream)
# with the C's 64-bit operations, against the reference carve() (maze_emu.ref).  python3 tools/maze_stream_emu.py
import os
import sys
import threading

import numpy as np

src = open(os.path.join(os.path.dirname(__file__), "maze_emu.py")).read()
exec(src.split("import threading")[0])  # perm_of, ref, ...
M64 = (1 << 64) - 1
PERIOD = 16


def nib(o):
    return (o & 3) | ((o >> 30) & 0xC)


def dbit(o, bp):
    return 1 if (o >> 11) * (1.0 / 9007199254740992.0) < bp else 0


def stream_groups(h, w):
    cells = ((w - 1) // 2) * ((h - 1) // 2)
    outputs = (9 * cells) // 5 + 64
    per_item = 32 * 8
    return (outputs + per_item - 1) // per_item * 8


class Win:
    pass


def dfs(seed, h, w, bp, ng):
    g = np.random.default_rng(seed).bit_generator
    N = ng * 32
    raw = [int(g.random_raw()) for _ in range(N)]  # the precomputed part; g continues past it (the overflow)
    H = [0] * ng
    D = [0] * ng
    for k, o in enumerate(raw):
        H[k >> 5] |= nib(o) << (4 * (k & 31))
        D[k >> 5] |= dbit(o, bp) << (k & 31)
    W = Win()
    W.h = 0  # 128-bit h1:h0
    W.d = 0
    W.avail = W.e = W.has32 = W.b2 = 0
    W.stage = (0, 0)  # (256-bit halves, 64-bit doubles) of groups e>>5, +1

    def stage(gq):
        hh = (H[gq] if gq < ng else 0) | ((H[gq + 1] if gq + 1 < ng else 0) << 128)
        dd = (D[gq] if gq < ng else 0) | ((D[gq + 1] if gq + 1 < ng else 0) << 32)
        W.stage = (hh, dd)

    def refill():
        need = 32 - W.avail
        if need <= 0:
            return
        off = W.e & 31
        t = (W.stage[0] >> (4 * off)) & ((1 << 128) - 1)
        td = (W.stage[1] >> off) & 0xFFFFFFFF
        ok = max(0, min(need, N - W.e))
        t &= (1 << (4 * ok)) - 1
        td &= (1 << ok) - 1
        W.h |= (t << (4 * W.avail)) & ((1 << 128) - 1)
        W.d |= (td << W.avail) & 0xFFFFFFFF
        for k in range(ok, need):
            o = int(g.random_raw())
            pos = W.avail + k
            W.h |= nib(o) << (4 * pos)
            W.d |= dbit(o, bp) << pos
        W.e += need
        W.avail = 32

    def shift(p):
        W.h >>= 4 * p
        W.d >>= p
        W.avail -= p

    def perm_draw(hs, u0):
        X = (((hs << 2) | W.b2) & M64) if W.has32 else hs
        rej = X & (X >> 1) & 0x5555555555555554
        kept = ~rej & 0x5555555555555554
        v = kept | (1 << 62)
        i2 = ((v & -v).bit_length() - 1) >> 1
        t = i2 + 2
        ic = min(i2, 30)
        pidx = (X & 3) * 6 + ((X >> (2 * ic)) & 3) * 2 + ((X >> (2 * ic + 2)) & 1)
        q = t - W.has32
        p = (q + 1) >> 1
        valid = 2 * (W.avail - u0) + W.has32
        return pidx, p, q, t <= min(valid, 32)

    ncx, ncy = (w - 1) // 2, (h - 1) // 2
    vis = np.zeros((ncy, ncx), bool)
    vis[0, 0] = True
    stack = []
    log = []
    stage(0)
    refill()
    stage(W.e >> 5)
    pidx, p, q, ok = perm_draw(W.h & M64, 0)
    assert ok
    W.has32 = q & 1
    W.b2 = ((W.h & M64) >> (4 * (p - 1) + 2)) & 3
    shift(p)
    perm = perm_of(pidx)
    cx = cy = k = 0
    frm = 0
    first = True
    done = False
    stalls = 0
    while not done:
        for _ in range(PERIOD):
            if done:
                continue
            E = 0
            if cx + 1 < ncx and not vis[cy, cx + 1]: E |= 1
            if cx - 1 >= 0 and not vis[cy, cx - 1]: E |= 2
            if cy + 1 < ncy and not vis[cy + 1, cx]: E |= 4
            if cy > 0 and not vis[cy - 1, cx]: E |= 8
            pm = 0
            for j in range(4): pm |= ((E >> ((perm >> (2 * j)) & 3)) & 1) << j
            pm &= (0xF << k) & 0xF
            j = (pm & -pm).bit_length() - 1 if pm else 4
            d = (perm >> (2 * j)) & 3 if pm else 0
            dneed = pm != 0 and not first
            carve = pm != 0 and (first or (W.d & 1) != 0)
            u0 = 1 if dneed else 0
            h0 = W.h & M64
            hs = ((h0 >> 4) | ((W.h >> 64) << 60)) & M64 if dneed else h0
            npx, p, q, ok = perm_draw(hs, u0)
            used = u0 + (p if carve else 0)
            if used > W.avail or (carve and not ok):
                assert W.avail < 32
                stalls += 1
                continue
            if carve:
                W.has32 = q & 1
                W.b2 = (hs >> (4 * (p - 1) + 2)) & 3
            shift(used)
            if pm:
                k = j + 1
            if carve:
                nx = cx + (d == 0) - (d == 1)
                ny = cy + (d == 2) - (d == 3)
                vis[ny, nx] = True
                log.append((nx, ny, d))
                stack.append((cx, cy, pidx, frm))
                cx, cy, frm, first, k, pidx = nx, ny, d, True, 0, npx
                perm = perm_of(pidx)
            elif pm == 0:
                if not stack:
                    done = True
                    continue
                child = frm
                cx, cy, pidx, frm = stack.pop()
                perm = perm_of(pidx)
                k = [((perm >> (2 * jj)) & 3) == child for jj in range(4)].index(True) + 1
                first = False
        # memory phase
        if not done:
            refill()
            stage(W.e >> 5)
    m = np.ones((h, w), bool)
    m[1, 1] = False
    for x, y, d in log:
        X, Y = 2 * x + 1, 2 * y + 1
        m[Y, X] = False
        m[Y - ((d == 2) - (d == 3)), X - ((d == 0) - (d == 1))] = False
    return m, stalls


def main():
    cases = [(21, 21, 1.0, None), (63, 63, 1.0, None), (127, 127, 1.0, None), (21, 35, 0.5, None), (127, 127, 0.3, None),
             (15, 9, 0.8, None), (3, 3, 1.0, None), (21, 21, 1.0, 8), (63, 63, 0.5, 8), (127, 127, 1.0, 8)]
    for h, w, bp, ng in cases:
        ngv = ng or stream_groups(h, w)
        st = 0
        for idx in [0, 1, 12345, 2**32 - 1]:
            a, s = dfs(idx, h, w, bp, ngv)
            b = ref(idx, h, w, bp)
            assert np.array_equal(a, b), (h, w, bp, ng, idx)
            st += s
        print(h, w, bp, "ng", ngv, "ok, stalls", st, flush=True)


threading.stack_size(512 * 1024 * 1024)
t = threading.Thread(target=main)
t.start()
t.join()
