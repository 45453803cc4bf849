"""Independent Python transcription of bwa's mem_chain + mem_chain_flt (src/bwamem.c; klib's
ks_introsort for the weight sort) -- the checker of oracle/chain_ref.c on small inputs.

Written against the same upstream semantics as the C oracle but with Python structures: chains
as dicts in a list kept sorted by start (kbtree stand-in with the same duplicate rule), the
introsort over a Python list by indices.  Slow; for a few hundred reads."""


def _test_and_merge(opt, l_pac, c, p):
    last = c["seeds"][-1]
    first = c["seeds"][0]
    qend, rend = last[1] + last[2], last[0] + last[2]
    if p[1] >= first[1] and p[1] + p[2] <= qend and p[0] >= first[0] and p[0] + p[2] <= rend:
        return True
    if (last[0] < l_pac or first[0] < l_pac) and p[0] >= l_pac:
        return False
    x, y = p[1] - last[1], p[0] - last[0]
    if y >= 0 and x - y <= opt["w"] and y - x <= opt["w"] and x - last[2] < opt["max_chain_gap"] and \
            y - last[2] < opt["max_chain_gap"]:
        c["seeds"].append(p)
        return True
    return False


def _weight(c):
    w, end = 0, 0
    for (rb, qb, ln) in c["seeds"]:
        if qb >= end:
            w += ln
        elif qb + ln > end:
            w += qb + ln - end
        end = max(end, qb + ln)
    tmp, w, end = w, 0, 0
    for (rb, qb, ln) in c["seeds"]:
        if rb >= end:
            w += ln
        elif rb + ln > end:
            w += rb + ln - end
        end = max(end, rb + ln)
    return min(min(w, tmp), (1 << 30) - 1)


def _insertsort(a, s, t, lt):
    for i in range(s + 1, t):
        j = i
        while j > s and lt(a[j], a[j - 1]):
            a[j], a[j - 1] = a[j - 1], a[j]
            j -= 1


def _combsort(a, s, n, lt):
    shrink = 1.2473309501039786540366528676643
    gap = n
    while True:
        if gap > 2:
            gap = int(gap / shrink)
            if gap in (9, 10):
                gap = 11
        swapped = False
        for i in range(s, s + n - gap):
            j = i + gap
            if lt(a[j], a[i]):
                a[i], a[j] = a[j], a[i]
                swapped = True
        if not (swapped or gap > 2):
            break
    if gap != 1:
        _insertsort(a, s, s + n, lt)


def introsort(a, lt):
    """klib ks_introsort on list a (indices for pointers)"""
    n = len(a)
    if n < 1:
        return
    if n == 2:
        if lt(a[1], a[0]):
            a[0], a[1] = a[1], a[0]
        return
    d = 2
    while (1 << d) < n:
        d += 1
    stack = []
    s, t = 0, n - 1
    d <<= 1
    while True:
        if s < t:
            d -= 1
            if d == 0:
                _combsort(a, s, t - s + 1, lt)
                t = s
                continue
            i, j = s, t
            k = i + ((j - i) >> 1) + 1
            if lt(a[k], a[i]):
                if lt(a[k], a[j]):
                    k = j
            else:
                k = i if lt(a[j], a[i]) else j
            rp = a[k]
            if k != t:
                a[k], a[t] = a[t], a[k]
            while True:
                i += 1
                while lt(a[i], rp):
                    i += 1
                j -= 1
                while i <= j and lt(rp, a[j]):
                    j -= 1
                if j <= i:
                    break
                a[i], a[j] = a[j], a[i]
            a[i], a[t] = a[t], a[i]
            if i - s > t - i:
                if i - s > 16:
                    stack.append((s, i - 1, d))
                s = i + 1 if t - i > 16 else t
            else:
                if t - i > 16:
                    stack.append((i + 1, t, d))
                t = i - 1 if i - s > 16 else s
        else:
            if not stack:
                _insertsort(a, 0, n, lt)
                return
            s, t, d = stack.pop()


def mem_chain_read(opt, sa, l_pac, read_len, mems):
    """one read: intervals (k, l, s, info) in info order -> kept chains [[(rbeg, qbeg, len), ...], ...]"""
    chains = []
    if read_len < opt["min_seed_len"]:
        return []
    for (k0, _l, s, info) in mems:
        slen = (info & 0xffffffff) - (info >> 32)
        step = s // opt["max_occ"] if s > opt["max_occ"] else 1
        k = count = 0
        while k < s and count < opt["max_occ"]:
            p = (int(sa[k0 + k]), info >> 32, slen)
            k += step
            count += 1
            if p[0] < l_pac < p[0] + p[2]:
                continue
            starts = [c["pos"] for c in chains]
            lo = next((i for i, x in enumerate(starts) if x >= p[0]), len(chains))
            eq = lo < len(chains) and starts[lo] == p[0]
            lower = lo if eq else lo - 1
            if lower >= 0 and _test_and_merge(opt, l_pac, chains[lower], p):
                continue
            chains.insert(lo + 1 if eq else lo, {"pos": p[0], "seeds": [p]})
    # mem_chain_flt
    a = []
    for c in chains:
        c["w"], c["kept"], c["first"] = _weight(c), 0, -1
        if c["w"] >= opt["min_chain_weight"]:
            a.append(c)
    if not a:
        return []
    introsort(a, lambda x, y: x["w"] > y["w"])
    beg = lambda c: c["seeds"][0][1]                           # noqa: E731
    end = lambda c: c["seeds"][-1][1] + c["seeds"][-1][2]      # noqa: E731
    a[0]["kept"] = 3
    kept = [0]
    for i in range(1, len(a)):
        large = False
        broke = False
        for j in kept:
            b_max, e_min = max(beg(a[j]), beg(a[i])), min(end(a[j]), end(a[i]))
            if e_min > b_max:
                min_l = min(end(a[i]) - beg(a[i]), end(a[j]) - beg(a[j]))
                if e_min - b_max >= min_l * opt["mask_level"] and min_l < opt["max_chain_gap"]:
                    large = True
                    if a[j]["first"] < 0:
                        a[j]["first"] = i
                    if a[i]["w"] < a[j]["w"] * opt["drop_ratio"] and a[j]["w"] - a[i]["w"] >= opt["min_seed_len"] << 1:
                        broke = True
                        break
        if not broke:
            kept.append(i)
            a[i]["kept"] = 2 if large else 3
    for j in kept:
        if a[j]["first"] >= 0:
            a[a[j]["first"]]["kept"] = 1
    k = 0
    i = 0
    while i < len(a):
        if a[i]["kept"] not in (0, 3):
            k += 1
            if k >= opt["max_chain_extend"]:
                break
        i += 1
    for i2 in range(i, len(a)):
        if a[i2]["kept"] < 3:
            a[i2]["kept"] = 0
    return [c["seeds"] for c in a if c["kept"] != 0]
