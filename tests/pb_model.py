"""Lane-by-lane model of cg_pcl.h pcl_block_sort (512 threads, PER elements each), with every
array access bounds-checked, for tests/test_pcl_block_model.py: the same steps, ballots and
index arithmetic as the device code, checked against libstdc++'s std::sort permutation
(cg_sort.h restated in Python: tests/pb_model.std_sort)."""

THRESH = 16
HEAD, FIN, DEPTH, SC_SHIFT, SC_MASK = 0x80000000, 0x40000000, 0xFF, 8, 0x7FF


class Arr:
    """Fixed-size array that raises on any access outside [0, n)."""

    def __init__(self, n, fill=0):
        self.v = [fill] * n

    def __getitem__(self, i):
        if not 0 <= i < len(self.v):
            raise IndexError(f"read {i} of {len(self.v)}")
        return self.v[i]

    def __setitem__(self, i, x):
        if not 0 <= i < len(self.v):
            raise IndexError(f"write {i} of {len(self.v)}")
        self.v[i] = x


def key(r):
    return r >> 32


# ---- libstdc++ std::sort (cg_sort.h restated) ----------------------------------------------
def _lg(n):
    r = 0
    while n > 1:
        n >>= 1
        r += 1
    return r


def _adjust_heap(f, base, hole, ln, value):
    top = hole
    second = hole
    while second < (ln - 1) // 2:
        second = 2 * (second + 1)
        if key(f[base + second]) < key(f[base + second - 1]):
            second -= 1
        f[base + hole] = f[base + second]
        hole = second
    if (ln & 1) == 0 and second == (ln - 2) // 2:
        second = 2 * (second + 1)
        f[base + hole] = f[base + second - 1]
        hole = second - 1
    parent = (hole - 1) // 2
    while hole > top and key(f[base + parent]) < key(value):
        f[base + hole] = f[base + parent]
        hole = parent
        parent = (hole - 1) // 2
    f[base + hole] = value


def heap_sort_range(f, base, ln):
    if ln >= 2:
        parent = (ln - 2) // 2
        while True:
            _adjust_heap(f, base, parent, ln, f[base + parent])
            if parent == 0:
                break
            parent -= 1
    while ln > 1:
        ln -= 1
        v = f[base + ln]
        f[base + ln] = f[base]
        _adjust_heap(f, base, 0, ln, v)


def move_median_to_first(f, result, a, b, c):
    def lt(i, j):
        return key(f[i]) < key(f[j])

    def sw(i, j):
        f[i], f[j] = f[j], f[i]

    if lt(a, b):
        if lt(b, c):
            sw(result, b)
        elif lt(a, c):
            sw(result, c)
        else:
            sw(result, a)
    elif lt(a, c):
        sw(result, a)
    elif lt(b, c):
        sw(result, c)
    else:
        sw(result, b)


def std_sort(a, depth0=None):
    """std::sort(a, a + n) by key; depth0 overrides the depth budget 2 * floor(log2 n)."""
    f = list(a)
    n = len(f)
    if n <= 1:
        return f
    stk = [(0, n, 2 * _lg(n) if depth0 is None else depth0)]
    while stk:
        first, last, depth = stk.pop()
        while last - first > THRESH:
            if depth == 0:
                heap_sort_range(f, first, last - first)
                break
            depth -= 1
            move_median_to_first(f, first, first + 1, first + (last - first) // 2, last - 1)
            lo, hi, p = first + 1, last, key(f[first])
            while True:
                while key(f[lo]) < p:
                    lo += 1
                hi -= 1
                while p < key(f[hi]):
                    hi -= 1
                if not lo < hi:
                    break
                f[lo], f[hi] = f[hi], f[lo]
                lo += 1
            stk.append((lo, last, depth))
            last = lo
    # insertion sort: stable by key
    return sorted(f, key=key)


# ---- the block model ------------------------------------------------------------------------
BLOCK, WAVES = 512, 8

PW_MAX = 64


def _popc(m):
    return bin(m).count("1")


# ---- the large path's partition levels (cg_large.hip lg_pq_split / lg_pq_swap / lg_pcl_leaf) ----
def _pb_median(a, b, c, ka, kb, kc):
    if ka < kb:
        return b if kb < kc else (c if ka < kc else a)
    if ka < kc:
        return a
    return c if kb < kc else b


def levels_sort(E_in, leaf=4096, levels=None):
    """cg_large.hip lg_pq_split / lg_pq_swap / lg_pcl_leaf: partition levels over the whole
    array (tile layout aside: the look-back becomes a prefix over the range), at most `levels`
    of them (None: until no range longer than `leaf` with budget left remains), then every leaf
    through block_sort (a longer one through std::sort with its budget); returns the records."""
    n = len(E_in)
    if levels is None:
        levels = 1 << 30
    bufs = [list(E_in), [None] * n]
    leaves = []
    cur = []
    d0 = 2 * _lg(n) if n else 0
    if n <= leaf or _lg(n) == 0:
        leaves.append((0, n, d0, 0))
    else:
        cur = [(0, n, d0)]
    for lv in range(levels):
        if not cur:
            break
        E, Eo = bufs[lv % 2], bufs[(lv + 1) % 2]
        nxt = []
        for (f, e, d) in cur:
            a, b, c = f + 1, f + (e - f) // 2, e - 1
            m = _pb_median(a, b, c, key(E[a]), key(E[b]), key(E[c]))
            p = key(E[m])

            def V(x):
                return E[f if x == m else (m if x == f else x)]
            PL = [x for x in range(f + 1, e) if key(V(x)) >= p]
            PRa = [x for x in range(f + 1, e) if key(V(x)) <= p]   # ascending
            gi = {x: i for i, x in enumerate(PL)}
            li = {x: i for i, x in enumerate(PRa)}
            nL, nR = len(PL), len(PRa)
            Eo[f] = E[m]
            cuts = []
            for x in range(f + 1, e):
                vx = V(x)
                ge, le = key(vx) >= p, key(vx) <= p
                partner = x
                if ge and gi[x] < nR:
                    g = gi[x]
                    j = PRa[nR - 1 - g]
                    if x < j:
                        partner = j
                        nxt_ok = g + 1 < min(nL, nR)
                        if not nxt_ok or not PL[g + 1] < PRa[nR - 2 - g]:
                            cuts.append(min(PL[g + 1] if g + 1 < nL else 0xFFFFFFFF, j))
                    elif g == 0:
                        cuts.append(x)
                if le:
                    ri = nR - 1 - li[x]
                    if ri < nL and PL[ri] < x:
                        assert partner == x
                        partner = PL[ri]
                Eo[x] = vx if partner == x else V(partner)
            assert len(cuts) == 1, cuts
            cut = cuts[0]
            for lo, hi in ((f, cut), (cut, e)):
                if hi - lo > leaf and d > 1 and lv < levels - 1:
                    nxt.append((lo, hi, d - 1))
                else:
                    leaves.append((lo, hi, d - 1, (lv + 1) % 2))
        cur = nxt
    assert not cur
    out = [None] * n
    for (f, e, d, b) in leaves:   # lg_pcl_leaf -> lg_pcl_mid (17-64 records: one wave each)
        seg = bufs[b][f:e]
        if e - f > min(leaf, 4096):
            out[f:e] = std_sort(seg, depth0=d)
            continue
        lo, mids = block_sort(seg, depth0=d, wmax=512, defer=True)
        for (mf, mm, md, mrecs) in mids:
            mo, waves = block_sort(mrecs, depth0=md, defer=True)
            for (wf, wm, wd, wrecs) in waves:
                mo[wf:wf + wm] = wave_sort(wrecs, wd)
            lo[mf:mf + mm] = mo
        assert None not in lo
        out[f:e] = lo
    return out


# ---- cg_pcl.h pw_range64: one wave sorts a range of at most 64 records in registers ---------
def wave_sort(recs, depth):
    """cg_pcl.h pw_range64, lane by lane: lane l holds record l and its sub-range [hd, en) and
    budget; every sub-range longer than 16 with budget partitions in the same round (lane
    tables PG / PL as ds_permute builds them, reads as ds_bpermute); spent budgets heapsort;
    then a stable rank inside each sub-range of at most 16 (heapsorted ones: as they are)."""
    m = len(recs)
    assert 16 < m <= 64
    L = range(64)
    v = [recs[l] if l < m else 0xFFFFFFFFFFFFFFFF for l in L]
    live = [l < m for l in L]
    hd = [0 if live[l] else l for l in L]
    en = [m if live[l] else l + 1 for l in L]
    dep = [depth] * 64

    def bperm(src, x):   # x of lane src (addresses wrap at 64 lanes)
        return [x[src[l] & 63] for l in L]

    def ballot(pred):
        return sum(1 << l for l in L if pred[l])

    def mbcnt(mask, l):
        return _popc(mask & ((1 << l) - 1))

    while True:
        act = [live[l] and en[l] - hd[l] > THRESH and dep[l] > 0 for l in L]
        if not any(act):
            break
        a = [hd[l] + 1 for l in L]
        b = [hd[l] + (en[l] - hd[l]) // 2 for l in L]
        c = [en[l] - 1 for l in L]
        k0 = [key(x) for x in v]
        ka, kb, kc = bperm(a, k0), bperm(b, k0), bperm(c, k0)
        kh = bperm(hd, k0)
        mi = [_pb_median(a[l], b[l], c[l], ka[l], kb[l], kc[l]) for l in L]
        p = [ka[l] if mi[l] == a[l] else (kb[l] if mi[l] == b[l] else kc[l]) for l in L]
        # __move_median_to_first, virtually: position mi holds the first's record (key kh)
        k = [kh[l] if act[l] and l == mi[l] else k0[l] for l in L]
        inn = [act[l] and l > hd[l] for l in L]
        GE = ballot([inn[l] and k[l] >= p[l] for l in L])
        LE = ballot([inn[l] and k[l] <= p[l] for l in L])
        lo = [(1 << (hd[l] + 1)) - 1 if hd[l] + 1 < 64 else (1 << 64) - 1 for l in L]
        hi = [(1 << en[l]) - 1 if en[l] < 64 else (1 << 64) - 1 for l in L]
        bG = [_popc(GE & lo[l]) for l in L]
        bL = [_popc(LE & lo[l]) for l in L]
        nL = [_popc(GE & hi[l]) - bG[l] for l in L]
        nR = [_popc(LE & hi[l]) - bL[l] for l in L]
        isG = [(GE >> l) & 1 == 1 for l in L]
        isL = [(LE >> l) & 1 == 1 for l in L]
        gk = [mbcnt(GE, l) - bG[l] for l in L]
        rk = [nR[l] - 1 - (mbcnt(LE, l) - bL[l]) for l in L]
        tG, tL = _popc(GE), _popc(LE)
        PG, PLt = [None] * 64, [None] * 64   # ds_permute: every lane pushes its id
        for l in L:
            dg = mbcnt(GE, l) if isG[l] else tG + mbcnt(~GE & ((1 << 64) - 1), l)
            dl = mbcnt(LE, l) if isL[l] else tL + mbcnt(~LE & ((1 << 64) - 1), l)
            assert PG[dg] is None and PLt[dl] is None
            PG[dg], PLt[dl] = l, l
        # R_r (a <= lane, reverse rank r) is swapped iff L_r < R_r, i.e. more than r >= lanes
        # precede it in the sub-range: the swap count is one ballot, no lane lookup
        SW = ballot([isL[l] and mbcnt(GE, l) - bG[l] > rk[l] for l in L])
        s = [_popc(SW & hi[l]) - _popc(SW & lo[l]) for l in L]
        Rk = bperm([bL[l] + nR[l] - 1 - gk[l] if isG[l] and gk[l] < s[l] else 0 for l in L], PLt)
        Lk = bperm([bG[l] + rk[l] if isL[l] and 0 <= rk[l] < s[l] else 0 for l in L], PG)
        partner = list(L)
        for l in L:
            if isG[l] and gk[l] < s[l]:
                partner[l] = Rk[l]
            if isL[l] and rk[l] < s[l]:
                assert partner[l] == l
                partner[l] = Lk[l]
        # the virtual records: position mi holds v[hd], position hd holds v[mi]
        src = [(hd[l] if partner[l] == mi[l] else (mi[l] if partner[l] == hd[l] else partner[l])) if act[l] else l
               for l in L]
        v = bperm(src, v)
        gc = bperm([bG[l] + (s[l] if s[l] < nL[l] else 0) for l in L], PG)
        lc = bperm([bL[l] + nR[l] - (s[l] if s[l] else nR[l]) for l in L], PLt)
        for l in L:
            if act[l]:
                cut = gc[l] if s[l] == 0 else min(gc[l] if s[l] < nL[l] else 64, lc[l])
                if l >= cut:
                    hd[l] = cut
                else:
                    en[l] = cut
                dep[l] -= 1
    heap = [live[l] and en[l] - hd[l] > THRESH for l in L]
    for l in L:
        if heap[l] and l == hd[l]:
            seg = v[hd[l]:en[l]]
            heap_sort_range(seg, 0, en[l] - hd[l])
            v[hd[l]:en[l]] = seg
    out = [None] * m
    for l in range(m):
        if heap[l]:
            rank = l - hd[l]
        else:
            kx = key(v[l])
            rank = sum(1 for j in range(hd[l], en[l]) if key(v[j]) < kx or (key(v[j]) == kx and j < l))
        out[hd[l] + rank] = v[l]
    return out


def block_sort(E_in, PER=None, depth0=None, oop=False, wmax=PW_MAX, defer=False):
    """cg_pcl.h pcl_block_sort, thread by thread (element x = tid + 512 k; oop: the swaps go to a
    second buffer, as in the frame kernel), three barrier steps per level: each element's range carries its own
    bounds and budget (registers), S1 computes the range's median of three itself (the swap
    with the first stays virtual: V(m) = E[f], V(f) = E[m]), S4's swaps write V of the partner
    and the range's cutter (the last swap's L element, or L_0 when there is none) stores the
    cut, S0 follows it. No heads step: a range's set-up (median, budget, task or heapsort) is
    read off its bounds by every element. Ranges of 17..wmax records with budget left leave
    the levels as tasks: sorted by wave_sort (PwInline), or, with defer, returned as (first,
    size, budget, records) with their output positions left None (PqDefer)."""
    n = len(E_in)
    if PER is None:
        PER = 1 if n <= 512 else 2 if n <= 1024 else 4 if n <= 2048 else 8
    assert n <= BLOCK * PER
    if depth0 is None:
        depth0 = 2 * _lg(n) if n else 0
    E = Arr(n)
    E.v = list(E_in)
    out = Arr(n, None)
    S = {k: Arr(n + 1) for k in ("RLO", "PL", "PR", "CUT")}
    T = range(BLOCK)
    rg = [[(0, n, depth0)] * PER for _ in T]   # each element's range (first, last, budget)

    def part_of(f, e, d):
        return e - f > THRESH and d > 0 and e - f > wmax

    while True:
        st = [[None] * PER for _ in T]
        anyp = False
        cnt = {}
        for k in range(PER):                         # S1: the range's pivot, >= / <=, counts
            ge = [False] * BLOCK
            le = [False] * BLOCK
            for t in T:
                x = t + BLOCK * k
                f, e, d = rg[t][k]
                part = x < n and part_of(f, e, d)
                m = p = kx = None
                if part:
                    a, b, c = f + 1, f + (e - f) // 2, e - 1
                    m = _pb_median(a, b, c, key(E[a]), key(E[b]), key(E[c]))
                    p = key(E[m])
                    kx = key(E[f]) if x == m else key(E[x])
                inn = part and x > f
                ge[t], le[t] = inn and kx >= p, inn and kx <= p
                st[t][k] = dict(part=part, inn=inn, m=m)
                anyp |= part
            for w in range(WAVES):
                gm = sum(1 << l for l in range(64) if ge[64 * w + l])
                lm = sum(1 << l for l in range(64) if le[64 * w + l])
                cnt[k * WAVES + w] = _popc(gm) | (_popc(lm) << 16)
                for l in range(64):
                    t = 64 * w + l
                    st[t][k].update(ge=ge[t], le=le[t], mg=_popc(gm & ((1 << l) - 1)), ml=_popc(lm & ((1 << l) - 1)))
        if not anyp:                                 # (the S1 barrier's OR)
            break
        NS = PER * WAVES                             # S2
        c = [cnt[j] for j in range(NS)]
        gex = [sum(c[i] & 0xFFFF for i in range(j)) for j in range(NS)]
        hex_ = [sum(c[i] >> 16 for i in range(j)) for j in range(NS)]
        S["RLO"] = Arr(n + 1, None)
        for t in T:
            w = t // 64
            for k in range(PER):
                x = t + BLOCK * k
                q = st[t][k]
                gx, lx = gex[k * WAVES + w] + q["mg"], hex_[k * WAVES + w] + q["ml"]
                q.update(gx=gx, lx=lx)
                if x < n:
                    S["RLO"][x] = (gx + q["ge"]) | ((lx + q["le"]) << 16)
                if q["ge"]:
                    S["PL"][gx] = x
                if q["le"]:
                    S["PR"][lx] = x
        S["CUT"] = Arr(n + 1, None)
        val = {}
        for t in T:                                  # S4: partners, V of the partner, the cut
            for k in range(PER):
                x = t + BLOCK * k
                f, e, d = rg[t][k]
                q = st[t][k]
                if not q["part"]:
                    continue
                m = q["m"]
                if not q["inn"]:                     # the first position takes the median's record
                    val[x] = E[m]
                    continue
                bf, be = S["RLO"][f], S["RLO"][e - 1]
                gf, lend = bf & 0xFFFF, be >> 16
                nL, nR = (be & 0xFFFF) - gf, lend - (bf >> 16)
                li, ri = q["gx"] - gf, lend - 1 - q["lx"]
                partner = x
                if q["ge"] and li < nR:
                    j = S["PR"][lend - 1 - li]       # R_li
                    if x < j:
                        partner = j
                        if li + 1 >= min(nL, nR) or not S["PL"][gf + li + 1] < S["PR"][lend - 2 - li]:
                            S["CUT"][f] = min(S["PL"][gf + li + 1] if li + 1 < nL else 0xFFFFFFFF, j)
                    elif li == 0:                    # no swap at all: the left scan stops at L_0
                        S["CUT"][f] = x
                if q["le"] and ri < nL:
                    i = S["PL"][gf + ri]             # L_ri
                    if i < x:
                        assert partner == x, "an element swapped twice"
                        partner = i
                val[x] = E[f] if partner == m else E[partner]
        if oop:
            E2 = Arr(n)
            E2.v = list(E.v)
            for x, v in val.items():
                E2[x] = v
            E = E2
        else:
            for x, v in val.items():
                E[x] = v
        for t in T:                                  # S0
            for k in range(PER):
                if st[t][k]["part"]:
                    x = t + BLOCK * k
                    f, e, d = rg[t][k]
                    cc = S["CUT"][f]
                    rg[t][k] = (f, cc, d - 1) if x < cc else (cc, e, d - 1)
    tasks = []
    for t in T:                                      # heads: tasks and heapsorts
        for k in range(PER):
            x = t + BLOCK * k
            f, e, d = rg[t][k]
            if x < n and x == f and e - f > THRESH:
                if d == 0:
                    heap_sort_range(E, f, e - f)
                    for j in range(f, e):
                        out[j] = E[j]
                else:
                    assert e - f <= wmax
                    tasks.append((f, e - f, d, [E[j] for j in range(f, e)]))
    for (f, m, d, recs) in tasks:
        if not defer:
            for i, r in enumerate(wave_sort(recs, d)):
                out[f + i] = r
    for t in T:                                      # final insertion passes
        for k in range(PER):
            x = t + BLOCK * k
            f, e, d = rg[t][k]
            if x < n and e - f <= THRESH:
                kx = key(E[x])
                rank = sum(1 for j in range(f, e) if key(E[j]) < kx or (key(E[j]) == kx and j < x))
                out[f + rank] = E[x]
    return (out.v, tasks) if defer else out.v
