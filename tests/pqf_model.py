"""Tile-by-tile model of cg_large.hip lg_pq_flow (the device-sized PCL partition as one dataflow
launch) for tests/test_pq_flow_model.py: the same ticket queue, 16-byte entries (both halves'
bit layouts), look-back counts, range words, inline / deferred swaps, cut word, the children's
shared slots (ch[]), the block reserved by a range's first tile, the records-in-leaves count that
ends the launch and the leaf list, with every array access bounds-checked
(pb_model.Arr). Workgroups are modelled as a pool that takes tickets in order; a random
scheduler interleaves their steps (split, wait, swap, push) so that ranges of different depths
run side by side as on the device. The leaves then go through std::sort's restatement with
their budgets (their in-LDS sort is modelled in pb_model.block_sort). Returns the records and
the statistics the kernel's design relies on (every ticket served, the records count reaching n
only when every record is in a leaf)."""
import random

from pb_model import Arr, _lg, _pb_median, key, std_sort

PQ_T = 512
CUT = 2048            # LG_PCL_CUT
LEAF = 4096           # LG_PCL_LEAF
TILE = 1 << 46        # PQ_RW_TILE
RW_N = (1 << 23) - 1  # PQ_RW_N
KIND_SWAP = 1 << 7
NOP = 1 << 6
SD_BASE = 39          # PQF_SD_BASE
M32 = 0xFFFFFFFF


def tiles(f, e):
    return (e - f - 1 + PQ_T - 1) // PQ_T


def flow_sort(E_in, grid=8, seed=0, depth_cap=0, defer_p=0.3):
    rng = random.Random(seed)
    n = len(E_in)
    d0 = 2 * _lg(n)
    bufs = [Arr(n), Arr(n)]
    for i, r in enumerate(E_in):
        bufs[0][i] = r
    leaflist = []          # pq_push(PQ_LEAFLIST): (first, last, budget, buffer)
    if n <= CUT:
        leaflist.append((0, n, d0, 0))
        return finish(n, bufs, leaflist), {"tickets": 0}
    T0 = tiles(0, n)
    cap = 2 * (2 * _lg(n) + 2) * (n // PQ_T + n // CUT + 2) + 1024
    ent = Arr(2 * cap)
    lb = Arr(cap)
    rw = Arr(cap)
    sd = Arr(cap)
    par = Arr(n + 2)
    cnt = Arr(n + 2)
    recL = Arr(n + 2)
    recR = Arr(n + 2)
    vst = Arr(n)
    hdr = [0, 0, 0]        # tickets handed out, queued past T0, records in leaves
    st = {"tickets": 0, "deferred": 0, "inline": 0, "ranges": 1, "max_depth": 0, "nops": 0}

    def entry(k, f, e, w2, tb):
        assert 0 <= k < cap
        assert ent[2 * k] == 0 and ent[2 * k + 1] == 0, "a ticket published twice"
        ent[2 * k] = (e << 32) | f
        ent[2 * k + 1] = (tb << 32) | w2

    def push_leaf(f, e, d, b):
        leaflist.append((f, e, d, b))

    # a workgroup is a generator: it yields when it waits (for an entry or a range word)
    def workgroup():
        while True:
            t = hdr[0]
            hdr[0] += 1
            st["tickets"] = max(st["tickets"], hdr[0])
            f, e, w2, tb = 0, n, d0 | (T0 << 16), 0   # (range 0: its swap slots at [T0, 2 T0))
            if t >= T0:
                if t >= cap:
                    return
                while True:
                    a, b = ent[2 * t], ent[2 * t + 1]
                    if a and b:
                        f, e, w2, tb = a & M32, a >> 32, b & M32, b >> 32
                        break
                    if hdr[2] >= n:
                        return
                    yield "entry"
            assert f < e <= n, (f, e)
            if w2 & NOP:
                st["nops"] += 1
                continue
            d, depth = w2 & 0x3F, (w2 >> 8) & 0xFF
            swap_entry = (w2 & KIND_SWAP) != 0
            q = (w2 >> 16) if swap_entry else t - tb
            off = 0 if swap_entry else w2 >> 16   # split entries: the range's swap slots at tb + off
            T = tiles(f, e)
            assert 0 <= q < T
            if not swap_entry and q == 0:   # the children block, reserved as the range starts
                base = 2 * T0 + hdr[1]
                hdr[1] += 2 * (T + 1)
                sd[tb] = sd[tb] + (min(base, cap) << SD_BASE)
            E, Eo = bufs[depth & 1], bufs[(depth + 1) & 1]
            a_, b_, c_ = f + 1, f + (e - f) // 2, e - 1
            m = _pb_median(a_, b_, c_, key(E[a_]), key(E[b_]), key(E[c_]))
            p = key(E[a_]) if m == a_ else (key(E[b_]) if m == b_ else key(E[c_]))
            rf = E[f]
            xs = [f + 1 + q * PQ_T + tid for tid in range(PQ_T)]
            valid = [x < e for x in xs]
            rx = [E[x] if v else E[f] for x, v in zip(xs, valid)]
            vx = [rf if x == m else r for x, r in zip(xs, rx)]
            handed = hdr[0]
            gi = [0] * PQ_T
            li = [0] * PQ_T
            if not swap_entry:
                k_ = [key(r) if v else 0 for r, v in zip(vx, valid)]
                ge = [v and k >= p for k, v in zip(k_, valid)]
                le = [v and k <= p for k, v in zip(k_, valid)]
                tg, tl = sum(ge), sum(le)
                # look-back: counts of the range's earlier tiles (their status words)
                while any(lb[j] == 0 for j in range(tb, t)):
                    yield "lookback"
                bg = sum((lb[j] >> 32) & 0x3FFFFFFF for j in range(tb, t))   # (PQ_ST_V: flags off)
                bl = sum(lb[j] & M32 for j in range(tb, t))
                lb[t] = (tg << 32) | tl | (1 << 62)   # (published; the model's flag bit)
                rg = rl = 0
                for i in range(PQ_T):
                    gi[i], li[i] = bg + rg, bl + rl
                    if ge[i]:
                        par[f + 1 + gi[i]] = xs[i]
                        recL[f + 1 + gi[i]] = vx[i]
                        rg += 1
                    if le[i]:
                        cnt[f + 1 + li[i]] = xs[i]
                        recR[f + 1 + li[i]] = vx[i]
                        rl += 1
                rw[tb] = rw[tb] + (TILE | (tg << 23) | tl)
                yield "split"
                inline = handed >= tb + T and rng.random() >= defer_p
                slot = tb + off + q           # the tile's swap slot
                if not inline:
                    for i in range(PQ_T):
                        if valid[i]:
                            vst[xs[i]] = (gi[i] << 32) | li[i]
                    if slot < cap:
                        entry(slot, f, e, (w2 & 0xFFFF) | KIND_SWAP | (q << 16), tb)
                    st["deferred"] += 1
                    continue
                if slot < cap:
                    entry(slot, 0, 1, NOP, 0)
                st["inline"] += 1
            else:
                for i in range(PQ_T):
                    if valid[i]:
                        rk = vst[xs[i]]
                        gi[i], li[i] = rk >> 32, rk & M32
            while (rw[tb] >> 46) < T:
                yield "rangeword"
            w_ = rw[tb]
            nL, nR = (w_ >> 23) & RW_N, w_ & RW_N
            tcut = 0                  # the tile's cut + 1 when its cutter is here
            if q == 0:
                Eo[f] = E[m]
            for i in range(PQ_T):
                x = xs[i]
                if not valid[i]:
                    continue
                k = key(vx[i])
                ge, le = k >= p, k <= p
                hasL = ge and gi[i] < nR
                nx = hasL and gi[i] + 1 < min(nL, nR)
                ri = (nR - 1 - li[i]) & M32
                hasR = le and ri < nL
                iR = f + 1 + (nR - 1 - gi[i] if hasL else 0)
                iL = f + 1 + (ri if hasR else 0)
                jj, rjj = cnt[iR], recR[iR]
                l2 = par[f + 1 + (gi[i] + 1 if gi[i] + 1 < nL else 0)]
                r2 = cnt[f + 1 + (nR - 2 - gi[i] if nx else 0)]
                il, ril = par[iL], recL[iL]
                rec, cutter, cut = vx[i], False, 0
                if hasL:
                    if x < jj:
                        rec = rjj
                        assert rjj == (rf if jj == m else E[jj]), "list record != the partner's"
                        if not nx or not l2 < r2:
                            cutter, cut = True, min(l2 if gi[i] + 1 < nL else M32, jj)
                    elif gi[i] == 0:
                        cutter, cut = True, x
                if hasR and il < x:
                    rec = ril
                    assert ril == (rf if il == m else E[il]), "list record != the partner's"
                Eo[x] = rec
                if cutter:
                    assert tcut == 0, "two cutters in a tile"
                    tcut = min(max(cut, f), e) + 1
            yield "swap"
            # one add per tile: count, and the cut from the cutter's tile; the base came first
            add = 1 | (tcut << 16)
            assert not (tcut and (sd[tb] >> 16) & 0x7FFFFF), "two cutters in a range"
            sd[tb] = sd[tb] + add
            tot = sd[tb]
            done = (tot & 0xFFFF) - 1
            base = (tot >> SD_BASE) & 0xFFFFFF
            ch = [None] * 10
            nch = 0
            if done == T - 1:
                cw = 0 if tot >> 63 else (tot >> 16) & 0x7FFFFF
                assert cw
                fits = base + 2 * (T + 1) <= cap
                cut = cw - 1
                lo, hi = (f, cut), (cut, e)
                used = placed = 0
                for cc in range(2):
                    tcc = tiles(lo[cc], hi[cc])
                    r_ = hi[cc] - lo[cc] > CUT and d > 1 and not (depth_cap and depth + 1 >= depth_cap) and fits
                    if r_:
                        ch[2 + 2 * nch] = lo[cc]
                        ch[3 + 2 * nch] = hi[cc]
                        ch[6 + nch] = tcc
                        used += tcc
                        nch += 1
                        st["ranges"] += 1
                    else:
                        push_leaf(lo[cc], hi[cc], d - 1, (depth + 1) & 1)
                        placed += hi[cc] - lo[cc]
                st["max_depth"] = max(st["max_depth"], depth + 1)
                ch[0], ch[1] = nch, base
                # the children's entries and the leaves' count in either order
                w2c = (d - 1) | ((depth + 1) << 8)
                order = [0, 1] if rng.random() < 0.5 else [1, 0]
                for step in order:
                    if step == 0:
                        hdr[2] += placed
                    else:
                        # split slots [base, base + T + 1): the children's tiles, then nops; swap
                        # slots [base + T + 1, base + 2 T + 2): the children's tiles publish their
                        # own, the rest are nops
                        for i in range(2 * (T + 1)):
                            k = base + i
                            if k >= cap:
                                break
                            if i < used:
                                cc = 1 if (nch == 2 and i >= ch[6]) else 0
                                fb = base + (ch[6] if cc else 0)
                                entry(k, ch[2 + 2 * cc], ch[3 + 2 * cc], w2c | ((T + 1) << 16), fb)
                            elif i < T + 1 or i >= T + 1 + used:
                                entry(k, 0, 1, NOP, 0)
                    yield "push"

    pool = [workgroup() for _ in range(grid)]
    live = list(pool)
    steps = 0
    while live:
        g = rng.choice(live)
        try:
            next(g)
        except StopIteration:
            live.remove(g)
        steps += 1
        assert steps < 50_000_000, "no progress"
    assert hdr[2] == n, hdr
    return finish(n, bufs, leaflist), st


def finish(n, bufs, leaflist):
    """Every leaf sorted with its budget from the buffer its depth left it in (lg_pcl_leaf); the
    leaves must tile [0, n) exactly."""
    out = [None] * n
    for (f, e, d, b) in leaflist:
        seg = [bufs[b][i] for i in range(f, e)]
        srt = std_sort(seg, depth0=d)
        for i in range(f, e):
            assert out[i] is None, "overlapping leaves"
            out[i] = srt[i - f]
    assert None not in out, "a position no leaf covers"
    return out
