"""Independent pure-Python restatement of the POA consensus spec (oracle/poa_oracle.c header),
used only to cross-check the C oracle on small cases (test infrastructure)."""
from __future__ import annotations

NEG = -(1 << 29)


def poa_consensus(seqs, match=2, mismatch=4, gap_open=4, gap_ext=2, band_b=10, band_f_permille=10, max_seqs=32,
                  max_nodes=32768, **_):
    O, E = gap_open, gap_ext
    base = {}            # node -> base (0 source, 1 sink)
    ins = {0: [], 1: []}  # node -> [[pred, weight], ...] in creation order
    aligned = {}          # node -> [nodes]
    order = []
    n_nodes = 2
    used = 0

    def add_edge(a, b):
        for e in ins[b]:
            if e[0] == a:
                e[1] += 1
                return
        ins[b].append([a, 1])

    for s in seqs:
        if used >= max_seqs:
            break
        m = len(s)
        if m < 1 or n_nodes - 2 + m > max_nodes:
            continue
        if n_nodes == 2:
            prev = 0
            order = [0]
            for k in range(m):
                x = n_nodes
                n_nodes += 1
                base[x] = int(s[k])
                ins[x] = []
                aligned[x] = []
                add_edge(prev, x)
                prev = x
                order.append(x)
            add_edge(prev, 1)
            order.append(1)
            used += 1
            continue
        w = band_b + band_f_permille * m // 1000
        H, G, code, lo, hi, mpos = {}, {}, {}, {}, {}, {}
        lo[0], hi[0] = 0, min(m, w)
        H[0] = {j: (0 if j == 0 else -(O + E * j)) for j in range(0, hi[0] + 1)}
        G[0] = {j: NEG for j in range(0, hi[0] + 1)}
        mpos[0] = 0
        for v in order[1:]:
            if v == 1:
                continue
            preds = [p for p, _ in ins[v]]
            c = max(mpos[p] for p in preds) + 1
            lo[v], hi[v] = max(0, c - w), min(m, c + w)
            H[v], G[v], code[v] = {}, {}, {}
            F = {}
            best, bj = NEG - 1, lo[v]
            for j in range(lo[v], hi[v] + 1):
                D, dp = NEG, 0
                if j >= 1:
                    for k, u in enumerate(preds):
                        if lo[u] <= j - 1 <= hi[u] and H[u][j - 1] > NEG:
                            cand = H[u][j - 1] + (match if base[v] == s[j - 1] and base[v] < 4 else -mismatch)
                            if cand > D:
                                D, dp = cand, k
                g, ep, ee = NEG, 0, 0
                for k, u in enumerate(preds):
                    if lo[u] <= j <= hi[u]:
                        a = NEG if H[u][j] <= NEG else H[u][j] - O - E
                        b = NEG if G[u][j] <= NEG else G[u][j] - E
                        val = max(a, b)
                        if val > g:
                            g, ep, ee = val, k, int(b > a)
                f, fx = NEG, 0
                if j - 1 >= lo[v]:
                    a = NEG if H[v][j - 1] <= NEG else H[v][j - 1] - O - E
                    b = NEG if F[j - 1] <= NEG else F[j - 1] - E
                    f, fx = max(a, b), int(b > a)
                h, src = D, 0
                if g > h:
                    h, src = g, 1
                if f > h:
                    h, src = f, 2
                h = max(h, NEG)
                H[v][j], G[v][j], F[j] = h, max(g, NEG), max(f, NEG)
                code[v][j] = (src, ee, fx, dp, ep)
                if h > best:
                    best, bj = h, j
            mpos[v] = bj
        ub, bs = -1, NEG
        for u, _ in ins[1]:
            if lo[u] <= m <= hi[u] and H[u][m] > NEG and (ub < 0 or H[u][m] > bs):
                ub, bs = u, H[u][m]
        if ub < 0:
            continue
        path = []
        v, j, state = ub, m, 0
        while True:
            if v == 0:
                path += [(1, -1, jj - 1) for jj in range(j, 0, -1)]
                break
            src, ee, fx, dp, ep = code[v][j]
            if state == 0:
                if src == 0:
                    path.append((0, v, j - 1))
                    v, j = ins[v][dp][0], j - 1
                else:
                    state = src
            elif state == 1:
                path.append((2, v, -1))
                state = 1 if ee else 0
                v = ins[v][ep][0]
            else:
                path.append((1, -1, j - 1))
                state = 2 if fx else 0
                j -= 1
        path.reverse()
        rank = {y: r for r, y in enumerate(order)}

        def block_end(y):
            return max([y] + aligned[y], key=lambda q: rank[q])

        prev, first_new = 0, n_nodes
        chains, cur = {}, None
        for kind, v, jj in path:
            x, anchor, new = -1, None, False
            if kind == 0:
                b = int(s[jj])
                if base[v] == b:
                    x = v
                else:
                    for y in aligned[v]:
                        if base[y] == b:
                            x = y
                            break
                    if x < 0:
                        anchor = block_end(v)
                        x = n_nodes
                        n_nodes += 1
                        base[x], ins[x], aligned[x] = b, [], []
                        members = [v] + aligned[v]
                        for y in members:
                            if len(aligned[y]) < 4:
                                aligned[y].append(x)
                            if len(aligned[x]) < 4:
                                aligned[x].append(y)
                        new = True
            elif kind == 1:
                x = n_nodes
                n_nodes += 1
                base[x], ins[x], aligned[x] = int(s[jj]), [], []
                anchor = cur if prev >= first_new else (0 if prev == 0 else block_end(prev))
                new = True
            if x < 0:
                continue
            if new:
                if kind == 1 and prev >= first_new:
                    chains[anchor].append(x)
                else:
                    chains[anchor] = [x]
                cur = anchor
            add_edge(prev, x)
            prev = x
        add_edge(prev, 1)
        new_order = []
        for y in order:
            new_order.append(y)
            new_order += chains.get(y, [])
        order = new_order
        used += 1
    if used == 0:
        return [], 0
    score, bp = {0: 0}, {}
    for v in order[1:]:
        bw, bsc, bu = -1, 0, -1
        for u, wt in ins[v]:
            if bu < 0 or wt > bw or (wt == bw and score[u] > bsc):
                bw, bsc, bu = wt, score[u], u
        bp[v], score[v] = bu, (bw + bsc if bu >= 0 else 0)
    out, v = [], bp[1]
    while v >= 2:
        out.append(base[v])
        v = bp[v]
    return out[::-1], used
