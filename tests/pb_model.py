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
ACT, FINB, BUDGET = 0x100, 0x200, 0xFF


def _popc(m):
    return bin(m).count("1")


def _setup(E, S, cf, ce, d):
    info, act = d, False
    if ce - cf > THRESH:
        if d == 0:
            heap_sort_range(E, cf, ce - cf)
            info |= FINB
        else:
            move_median_to_first(E, cf, cf + 1, cf + (ce - cf) // 2, ce - 1)
            S["PIV"][cf] = key(E[cf])
            info |= ACT
            act = True
    S["INFO"][cf] = info
    return act


def block_sort(E_in, PER=None, depth0=None, oop=False):
    """cg_pcl.h pcl_block_sort, thread by thread: element x = tid + 512 k (oop: the swaps go
    to a second buffer, as in the frame kernel)."""
    n = len(E_in)
    if PER is None:
        PER = 1 if n <= 512 else 2 if n <= 1024 else 4 if n <= 2048 else 8
    assert n <= BLOCK * PER
    if depth0 is None:
        depth0 = 2 * _lg(n) if n else 0
    E = Arr(n)
    E.v = list(E_in)
    out = Arr(n)
    S = {k: Arr(n + 1) for k in ("INFO", "PIV", "RLO", "PL", "PR", "CUT")}
    cnt = Arr(8 * PER)
    MS = Arr(2 * 8 * PER)
    T = range(BLOCK)
    fe = [[n << 16] * PER for _ in T]
    anyact = _setup(E, S, 0, n, depth0) if n else False
    while anyact:
        st = [[0] * PER for _ in T]
        nn = [[0] * PER for _ in T]
        for k in range(PER):                         # S1
            ge = [False] * BLOCK
            le = [False] * BLOCK
            for t in T:
                x, f = t + BLOCK * k, fe[t][k] & 0xFFFF
                info = p = kx = 0
                if x < n:
                    info, p, kx = S["INFO"][f], S["PIV"][f], key(E[x])
                part = bool(info & ACT)
                inn = part and x > f
                ge[t], le[t] = inn and kx >= p, inn and kx <= p
                st[t][k] = dict(part=part, inn=inn)
            for w in range(WAVES):
                gm = sum(1 << l for l in range(64) if ge[64 * w + l])
                lm = sum(1 << l for l in range(64) if le[64 * w + l])
                cnt[k * WAVES + w] = _popc(gm) | (_popc(lm) << 16)
                MS[2 * (k * WAVES + w)], MS[2 * (k * WAVES + w) + 1] = gm, lm
                for l in range(64):
                    t = 64 * w + l
                    st[t][k].update(ge=ge[t], le=le[t], mg=_popc(gm & ((1 << l) - 1)), ml=_popc(lm & ((1 << l) - 1)))
        NS = PER * WAVES                             # S2: counts from the slot masks
        c = [cnt[j] for j in range(NS)]
        gex = [sum(c[i] & 0xFFFF for i in range(j)) for j in range(NS)]
        hex_ = [sum(c[i] >> 16 for i in range(j)) for j in range(NS)]
        totg, totl = sum(v & 0xFFFF for v in c), sum(v >> 16 for v in c)

        def before(y):   # (>= count, <= count) of the positions before y
            if (y >> 6) >= NS:
                return totg, totl
            sl, b = y >> 6, (1 << (y & 63)) - 1
            return gex[sl] + _popc(MS[2 * sl] & b), hex_[sl] + _popc(MS[2 * sl + 1] & b)
        for t in T:
            w = t // 64
            for k in range(PER):
                x, f, e = t + BLOCK * k, fe[t][k] & 0xFFFF, fe[t][k] >> 16
                q = st[t][k]
                gx, lx = gex[k * WAVES + w] + q["mg"], hex_[k * WAVES + w] + q["ml"]
                assert gx < 4096 and lx < 4096
                q.update(gx=gx, lx=lx)
                if q["part"]:
                    gf, lf = before(f + 1)
                    gend, lend = before(e)
                    nn[t][k] = (gend - gf, lend - lf)
                    if x == f:
                        S["CUT"][f] = 0
                    if q["inn"]:
                        li, ri = gx - gf, lend - lx - 1
                        if q["ge"]:
                            S["PL"][f + 1 + li] = x
                        if q["le"]:
                            S["PR"][f + 1 + ri] = x
                        q.update(li=li, ri=ri)
        val = {}
        for t in T:                                  # S4
            for k in range(PER):
                x, f = t + BLOCK * k, fe[t][k] & 0xFFFF
                q = st[t][k]
                if q["inn"]:
                    nL, nR = nn[t][k]
                    partner = x
                    if q["ge"] and q["li"] < nR:
                        j = S["PR"][f + 1 + q["li"]]
                        if x < j:
                            partner = j
                            li = q["li"]
                            if li + 1 >= min(nL, nR) or not S["PL"][f + 2 + li] < S["PR"][f + 2 + li]:
                                S["CUT"][f] = li + 1
                    if q["le"] and q["ri"] < nL:
                        i = S["PL"][f + 1 + q["ri"]]
                        if i < x:
                            assert partner == x, "an element swapped twice"
                            partner = i
                    if partner != x:
                        val[x] = E[partner]
        if oop:   # every record to the other buffer, then the buffers trade places
            E2 = Arr(n)
            E2.v = list(E.v)
            for x, v in val.items():
                E2[x] = v
            E = E2
        else:
            for x, v in val.items():
                E[x] = v
        anyact = False                               # S5
        for t in T:
            for k in range(PER):
                x, f, e = t + BLOCK * k, fe[t][k] & 0xFFFF, fe[t][k] >> 16
                if st[t][k]["part"] and x == f:
                    s, nL = S["CUT"][f], nn[t][k][0]
                    cut = S["PL"][f + 1] if s == 0 else min(S["PL"][f + 1 + s] if s < nL else 0xFFFFFFFF, S["PR"][f + s])
                    d = (S["INFO"][f] & BUDGET) - 1
                    anyact |= _setup(E, S, f, cut, d)
                    anyact |= _setup(E, S, cut, e, d)
                    S["CUT"][f] = cut
        for t in T:                                  # S0
            for k in range(PER):
                x, f, e = t + BLOCK * k, fe[t][k] & 0xFFFF, fe[t][k] >> 16
                if st[t][k]["part"]:
                    cc = S["CUT"][f]
                    fe[t][k] = (f | (cc << 16)) if x < cc else (cc | (e << 16))
    for t in T:
        for k in range(PER):
            x, f, e = t + BLOCK * k, fe[t][k] & 0xFFFF, fe[t][k] >> 16
            if x < n:
                r = E[x]
                if S["INFO"][f] & FINB:
                    out[x] = r
                else:
                    assert e - f <= THRESH
                    kx = key(r)
                    rank = sum(1 for j in range(f, e) if key(E[j]) < kx or (key(E[j]) == kx and j < x))
                    out[f + rank] = r
    return out.v


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
    for (f, e, d, b) in leaves:
        seg = bufs[b][f:e]
        out[f:e] = block_sort(seg, depth0=d) if e - f <= min(leaf, 4096) else std_sort(seg, depth0=d)
    return out


# ---- cg_pcl.h pw_range64: one wave sorts a range of at most 64 records in registers ---------
def _sel(mask, j):
    """Position of the j-th (0-based) set bit of a 64-bit mask: the popcount binary search."""
    lo = 0
    for step in (32, 16, 8, 4, 2, 1):
        if _popc(mask & ((1 << (lo + step)) - 1)) <= j:
            lo += step
    return lo


def wave64_sort(recs, depth):
    """The whole range [0, m) as __introsort_loop + __final_insertion_sort restricted to it
    (depth: the budget left on its path), lane i holding record i."""
    m = len(recs)
    assert m <= 64
    v = list(recs) + [None] * (64 - m)
    key_ = lambda i: key(v[i])
    stack = [(0, m, depth)]
    while stack:
        lo, hi, dep = stack.pop()
        while hi - lo > THRESH:
            if dep == 0:
                seg = v[lo:hi]
                heap_sort_range(seg, 0, hi - lo)
                v[lo:hi] = seg
                break
            dep -= 1
            a, b, c = lo + 1, lo + (hi - lo) // 2, hi - 1
            mi = _pb_median(a, b, c, key_(a), key_(b), key_(c))
            v[lo], v[mi] = v[mi], v[lo]
            p = key_(lo)
            GE = sum(1 << i for i in range(lo + 1, hi) if key_(i) >= p)
            LE = sum(1 << i for i in range(lo + 1, hi) if key_(i) <= p)
            nL, nR = _popc(GE), _popc(LE)
            # swap k pairs L_k (k-th set bit of GE) with R_k (the (nR-1-k)-th set bit of LE)
            s = sum(1 for k in range(min(nL, nR)) if _sel(GE, k) < _sel(LE, nR - 1 - k))
            nv = list(v)
            for i in range(lo + 1, hi):
                partner = i
                if (GE >> i) & 1:
                    k = _popc(GE & ((1 << i) - 1))
                    if k < s:
                        partner = _sel(LE, nR - 1 - k)
                if (LE >> i) & 1:
                    r = nR - 1 - _popc(LE & ((1 << i) - 1))
                    if r < s:
                        assert partner == i
                        partner = _sel(GE, r)
                nv[i] = v[partner]
            v = nv
            cut = _sel(GE, 0) if s == 0 else min(_sel(GE, s) if s < nL else 1 << 30, _sel(LE, nR - s))
            stack.append((cut, hi, dep))
            hi = cut
    # the final insertion passes: a stable rank over the whole (weakly ordered) range
    out = [None] * m
    for i in range(m):
        r = sum(1 for j in range(m) if key_(j) < key_(i) or (key_(j) == key_(i) and j < i))
        out[r] = v[i]
    return out
