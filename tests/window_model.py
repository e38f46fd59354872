"""Python model of the segmented long-piece tier's window rounds (kernels.hip bpe_wave_seg,
Tables::window) -- test infrastructure: tests/test_window_rule.py checks it against the
sequential merge loop of the reference (oracle/ref_py.py RefTokenizer.bpe, src/bpe.rs:88-153).

A round: r = the lowest rank of any pair; every site of r merges ((x, x) runs: the 1st, 3rd, ...
site), and so does the pair c = (x, y) of rank rc > r when c is the only minimum of its group of
positions and every other group overlapping its window [pos(c) - left(x), end(y) + right(y))
has a larger minimum.  Positions are the initial tokens' indices (fixed: a merged token keeps its
left position), groups are G = SW / 4 consecutive positions (SW = the per-lane segment width)."""


def window_meta(tok):
    """left(id) / right(id): the longest left side of a merge whose right side is id / right side
    of a merge whose left side is id, in chars (= bytes); None when the table is not eligible."""
    ranks, new_ids, id2s = tok.merge_ranks, tok.merge_new_ids, tok.id_to_token_map
    left, right = {}, {}
    for (a, b), r in ranks.items():
        if r >= len(new_ids):
            continue
        if len(id2s[new_ids[r]]) != len(id2s[a]) + len(id2s[b]):
            return None
        left[b] = max(left.get(b, 0), len(id2s[a]))
        right[a] = max(right.get(a, 0), len(id2s[b]))
    return left, right


def eager_set(tok):
    """Ranks whose merge is "eager" (ctok_host.cpp, Tables::eager): a merge consuming its token ranks
    before it.  Empty for a rank-monotone table."""
    INF = 1 << 62
    ranks, new_ids = tok.merge_ranks, tok.merge_new_ids
    mincons = {}
    for (a, b), r in ranks.items():
        if r < len(new_ids):
            for c in (a, b):
                mincons[c] = min(mincons.get(c, INF), r)
    return {r for r in ranks.values() if r < len(new_ids) and mincons.get(new_ids[r], INF) < r}


def _rank_sites(tok, t, rk, r, eager):
    """The sites of rank r one round applies (kernels.hip): every one ((x, x) runs: 1st, 3rd, ...),
    or for an eager merge the sites up to the first whose sequential new pairs rank below r
    (first_cascade; (x, x): the leftmost alone)."""
    ranks, new_ids = tok.merge_ranks, tok.merge_new_ids
    INF = 1 << 62
    n = len(t)
    sites = [i for i in range(n - 1) if rk[i] == r]
    fire = [False] * max(n - 1, 0)
    chain = t[sites[0]] == t[sites[0] + 1]
    if r in eager:
        if chain:
            fire[sites[0]] = True
            return fire
        nid = new_ids[r]
        for p in sites:
            fire[p] = True
            left_site = p >= 2 and fire[p - 2]
            rl = ranks.get((nid if left_site else t[p - 1], nid), INF) if p > 0 else INF
            rr = ranks.get((nid, t[p + 2]), INF) if p + 2 < n else INF
            if rl < r or rr < r:
                break
        return fire
    i = 0
    while i < n - 1:
        if rk[i] == r:
            j = i
            while j + 1 < n - 1 and rk[j + 1] == r:
                j += 1
            for q in range(i, j + 1, 2 if chain else 1):
                fire[q] = True
            i = j + 1
        else:
            i += 1
    return fire


def seg_width(m, k):
    return min(k, (((m + 63) // 64) + 15) & ~15)


def window_bpe(tok, ids, k=64, max_groups=16, eager=None, eager_ext=True):
    """The window rounds on one piece's initial ids; returns (ids, rounds).  `eager`: eager_set(tok)
    (computed when None) -- a candidate whose merge is eager never fires early."""
    INF = 1 << 62
    left, right = window_meta(tok)
    eager = eager_set(tok) if eager is None else eager
    ranks, new_ids = tok.merge_ranks, tok.merge_new_ids
    m = len(ids)
    g_w = seg_width(m, k) // 4
    t, pos = list(ids), list(range(m))
    rounds = 0
    while True:
        n = len(t)
        rk = [ranks.get((t[i], t[i + 1]), INF) for i in range(n - 1)]
        if not rk or min(rk) == INF:
            return t, rounds
        rounds += 1
        r = min(rk)
        fire = _rank_sites(tok, t, rk, r, eager)
        n_groups = (m + g_w - 1) // g_w
        gmin, gcnt, garg = [INF] * n_groups, [0] * n_groups, [None] * n_groups
        for i in range(n - 1):
            g = pos[i] // g_w
            if rk[i] < gmin[g]:
                gmin[g], gcnt[g], garg[g] = rk[i], 1, i
            elif rk[i] == gmin[g]:
                gcnt[g] += 1
        for g in range(n_groups):
            if gmin[g] in (INF, r) or gcnt[g] != 1:
                continue
            i = garg[g]
            lo = max(0, pos[i] - left.get(t[i], 0))
            end = min((pos[i + 2] if i + 2 < n else m) + right.get(t[i + 1], 0), m)
            if gmin[g] in eager:
                # an eager candidate (a merge consuming its token ranks below it): its new pairs
                # with today's neighbours must rank above it, and the window widens to the
                # neighbours' own windows, so that neither neighbour can change before its turn
                if not eager_ext:
                    continue
                nid = new_ids[gmin[g]]
                if (i > 0 and ranks.get((t[i - 1], nid), INF) <= gmin[g]) or \
                        (i + 2 < n and ranks.get((nid, t[i + 2]), INF) <= gmin[g]):
                    continue
                if i > 0:
                    lo = max(0, min(lo, pos[i - 1] - left.get(t[i - 1], 0)))
                if i + 2 < n:
                    end = min(max(end, (pos[i + 3] if i + 3 < n else m) + right.get(t[i + 2], 0)), m)
            h0, h1 = lo // g_w, (end - 1) // g_w
            if h1 - h0 >= max_groups:
                continue
            if all(gmin[h] > rk[i] for h in range(h0, h1 + 1) if h != g):
                fire[i] = True
        nt, npos, i = [], [], 0
        while i < n:
            if i < n - 1 and fire[i]:
                nt.append(new_ids[rk[i]])
                npos.append(pos[i])
                i += 2
            else:
                nt.append(t[i])
                npos.append(pos[i])
                i += 1
        t, pos = nt, npos


def window_bpe_dense(tok, ids, eager=None):
    """The dense (<= 256 B) tier's window rounds: local minima only, the window scanned outward
    from the pair over the tokens' first initial positions (kernels.hip bpe_wave_dense)."""
    INF = 1 << 62
    left, right = window_meta(tok)
    eager = eager_set(tok) if eager is None else eager
    ranks, new_ids = tok.merge_ranks, tok.merge_new_ids
    m0 = len(ids)
    t, pos = list(ids), list(range(m0))
    rounds = 0
    while True:
        n = len(t)
        rk = [ranks.get((t[i], t[i + 1]), INF) for i in range(n - 1)] + [INF]
        r = min(rk)
        if r == INF:
            return t, rounds
        rounds += 1
        fire = _rank_sites(tok, t, rk[:-1], r, eager) + [False]
        for p in range(n - 1):
            rc = rk[p]
            if rc in (INF, r) or (p > 0 and rk[p - 1] <= rc) or rk[p + 1] <= rc or rc in eager:
                continue
            lo = max(0, pos[p] - left.get(t[p], 0))
            hi = (pos[p + 2] if p + 2 < n else m0) + right.get(t[p + 1], 0)
            ok = True
            j = p
            while ok and j > 0:
                j -= 1
                if pos[j] < lo:
                    break
                ok = rk[j] > rc
            j = p + 1
            while ok and j + 1 < n:
                if pos[j] >= hi:
                    break
                ok = rk[j] > rc
                j += 1
            fire[p] = fire[p] or ok
        nt, npos, i = [], [], 0
        while i < n:
            if i < n - 1 and fire[i]:
                nt.append(new_ids[rk[i]])
                npos.append(pos[i])
                i += 2
            else:
                nt.append(t[i])
                npos.append(pos[i])
                i += 1
        t, pos = nt, npos
