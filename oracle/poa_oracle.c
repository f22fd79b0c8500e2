/*
 * poa_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker), never shipped.
 *
 * CPU restatement of the engine's allele-consensus mode: a banded partial-order
 * alignment (POA) consensus of the inserted sequences that support a refined INS call.
 * The north star names "abPOA banded partial-order consensus"; the reference declares
 * abPOA as a submodule (.gitmodules:4-6) but never includes or calls it (Makefile:16 links
 * -lhts -lz -pthread only), and the abPOA sources are absent from /root/reference.  So
 * there is NO reference behaviour: this restates abPOA's published algorithm (Gao et al.,
 * Bioinformatics 2021: global POA of each sequence against the graph with an adaptive band
 * of width b + f*len around the predecessors' best cells, graph fusion of matching bases,
 * heaviest-bundle consensus) with the engine's exact tie rules, and PARITY IS UNPINNED --
 * the GPU kernel is checked against this file, nothing checks this file against abPOA.
 *
 * Spec (the GPU kernel implements the same):
 *   score(a, b) = a == b && a < 4 ? +match : -mismatch       (nt4 codes, 4 = N)
 *   gap of length L = -(gap_open + L * gap_ext)               (affine)
 *   graph: node 0 = source, node 1 = sink, others carry one base; in-edges per node in
 *          creation order with weights; "aligned" groups of alternative bases.
 *   align S (length m) to the graph in topological order (source first):
 *     band(source) = [0, min(m, w)], w = band_b + band_f * m / 1000;
 *     band(v) = [max(0, c - w), min(m, c + w)], c = 1 + max over preds u of mpos[u];
 *     H[src][0] = 0, H[src][j] = F[src][j] = -(O + E j);
 *     D  = max_u H[u][j-1] + score(base v, S[j-1])            (j >= 1, j-1 in band u)
 *     Eg = max_u max(H[u][j] - O - E, Eg[u][j] - E)          (node v deleted; open on ties)
 *     F  = max(H[v][j-1] - O - E, F[v][j-1] - E)              (S[j-1] inserted; open on ties)
 *     H  = max(D, Eg, F), ties in that order; preds in in-edge order, first max wins;
 *     mpos[v] = smallest j of max H[v][.]
 *   end: first pred u of the sink (in-edge order) with m in band(u) and max H[u][m];
 *     none -> the sequence is skipped.  Traceback to the source, leading characters left
 *     at the source are insertions.
 *   fusion (forward along the path): a match to v reuses v if the base agrees, else the
 *     node of v's aligned group with that base, else a new node joining the group; an
 *     insertion makes a new node; a deletion adds nothing; edge prev->x gains weight 1
 *     (created if absent); finally last->sink.
 *   order: a topological order in which aligned groups are contiguous (see fuse); the DP
 *     values, tie choices and consensus do not depend on which topological order is used.
 *   sequences: in support order, the first starts the graph; a sequence is skipped when
 *     n_nodes + m > max_nodes; at most max_seqs are used.
 *   consensus (heaviest bundle): for each node in order, the in-edge with the largest
 *     (weight, score[pred]), first on ties; score[v] = weight + score[pred]; follow the
 *     choices back from the sink.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "svtrek_oracle.h"

#define NEG_INF (-(1 << 29))
#define POA_MAX_IN 64
#define POA_MAX_ALIGNED 4

typedef struct {
    int32_t n, cap;   /* nodes: 0 source, 1 sink */
    uint8_t *base;
    int32_t *nin;
    int32_t *in_pred;   /* [cap][POA_MAX_IN] */
    int32_t *in_w;
    int32_t *nal;
    int32_t *al;        /* [cap][POA_MAX_ALIGNED] */
    int32_t *ord;       /* topological order (node ids) */
    int32_t nord;
} graph_t;

static int g_init(graph_t *g, int cap) {
    memset(g, 0, sizeof *g);
    g->cap = cap;
    g->base = (uint8_t *)calloc((size_t)cap, 1);
    g->nin = (int32_t *)calloc((size_t)cap, 4);
    g->in_pred = (int32_t *)calloc((size_t)cap * POA_MAX_IN, 4);
    g->in_w = (int32_t *)calloc((size_t)cap * POA_MAX_IN, 4);
    g->nal = (int32_t *)calloc((size_t)cap, 4);
    g->al = (int32_t *)calloc((size_t)cap * POA_MAX_ALIGNED, 4);
    g->ord = (int32_t *)calloc((size_t)cap, 4);
    if (!g->base || !g->nin || !g->in_pred || !g->in_w || !g->nal || !g->al || !g->ord) return -1;
    g->n = 2;   /* source, sink */
    return 0;
}

static void g_free(graph_t *g) {
    free(g->base); free(g->nin); free(g->in_pred); free(g->in_w); free(g->nal); free(g->al); free(g->ord);
}

static void add_edge(graph_t *g, int from, int to) {
    int32_t *p = g->in_pred + (size_t)to * POA_MAX_IN, *w = g->in_w + (size_t)to * POA_MAX_IN;
    for (int k = 0; k < g->nin[to]; k++)
        if (p[k] == from) { w[k]++; return; }
    if (g->nin[to] < POA_MAX_IN) { p[g->nin[to]] = from; w[g->nin[to]] = 1; g->nin[to]++; }
}

static int new_node(graph_t *g, uint8_t b) {
    int x = g->n++;
    g->base[x] = b;
    g->nin[x] = 0;
    g->nal[x] = 0;
    return x;
}

static void join_group(graph_t *g, int v, int x) {
    /* x joins v's aligned group: every member learns x, x learns every member */
    int members[POA_MAX_ALIGNED + 1], nm = 0;
    members[nm++] = v;
    for (int k = 0; k < g->nal[v]; k++) members[nm++] = g->al[(size_t)v * POA_MAX_ALIGNED + k];
    for (int k = 0; k < nm; k++) {
        int y = members[k];
        if (g->nal[y] < POA_MAX_ALIGNED) g->al[(size_t)y * POA_MAX_ALIGNED + g->nal[y]++] = x;
        if (g->nal[x] < POA_MAX_ALIGNED) g->al[(size_t)x * POA_MAX_ALIGNED + g->nal[x]++] = y;
    }
}

static inline int sc(uint8_t a, uint8_t b, const orc_poa_params *pp) {
    return (a == b && a < 4) ? pp->match : -pp->mismatch;
}

/* path step: kind 0 = match (node, j), 1 = insertion (j), 2 = deletion (node) */
typedef struct { int32_t kind, node, j; } step_t;

/* Align s[0..m) to g; on success fills path (forward order) and returns its length, else -1. */
static int align(const graph_t *g, const uint8_t *s, int m, const orc_poa_params *pp, step_t *path,
                 int32_t *H, int32_t *Eg, int32_t *F, uint16_t *code, int32_t *lo, int32_t *hi,
                 int32_t *mpos, int32_t *rank, int W) {
    const int O = pp->gap_open, E = pp->gap_ext;
    const int w = pp->band_b + (int)((int64_t)pp->band_f_permille * m / 1000);
    for (int r = 0; r < g->nord; r++) rank[g->ord[r]] = r;
    /* source row */
    {
        const int v = 0;
        lo[v] = 0; hi[v] = m < w ? m : w;
        int32_t *h = H + (size_t)v * W, *e = Eg + (size_t)v * W, *f = F + (size_t)v * W;
        for (int j = lo[v]; j <= hi[v]; j++) {
            int t = j - lo[v];
            h[t] = j == 0 ? 0 : -(O + E * j);
            e[t] = NEG_INF;
            f[t] = j == 0 ? NEG_INF : h[t];
            code[(size_t)v * W + t] = (uint16_t)(j == 0 ? 0 : (2u | (j >= 2 ? 8u : 0u)));
        }
        mpos[v] = 0;
    }
    for (int r = 1; r < g->nord; r++) {
        const int v = g->ord[r];
        if (v == 1) continue;   /* sink: no row */
        const int np = g->nin[v];
        const int32_t *pr = g->in_pred + (size_t)v * POA_MAX_IN;
        int c = mpos[pr[0]];   /* every node but the source has a predecessor */
        for (int k = 1; k < np; k++) if (mpos[pr[k]] > c) c = mpos[pr[k]];
        c += 1;
        lo[v] = c - w < 0 ? 0 : c - w;
        hi[v] = c + w > m ? m : c + w;
        int32_t *h = H + (size_t)v * W, *e = Eg + (size_t)v * W, *f = F + (size_t)v * W;
        int best = NEG_INF - 1, bj = lo[v];
        for (int j = lo[v]; j <= hi[v]; j++) {
            const int t = j - lo[v];
            int D = NEG_INF, dp = 0;
            if (j >= 1) {
                for (int k = 0; k < np; k++) {
                    const int u = pr[k];
                    if (j - 1 < lo[u] || j - 1 > hi[u]) continue;
                    const int hv = H[(size_t)u * W + (j - 1 - lo[u])];
                    if (hv <= NEG_INF) continue;
                    const int cand = hv + sc(g->base[v], s[j - 1], pp);
                    if (cand > D) { D = cand; dp = k; }
                }
            }
            int G = NEG_INF, ep = 0, eext = 0;
            for (int k = 0; k < np; k++) {
                const int u = pr[k];
                if (j < lo[u] || j > hi[u]) continue;
                const int hv = H[(size_t)u * W + (j - lo[u])], ev = Eg[(size_t)u * W + (j - lo[u])];
                const int a = hv <= NEG_INF ? NEG_INF : hv - O - E;
                const int b = ev <= NEG_INF ? NEG_INF : ev - E;
                const int val = b > a ? b : a;
                if (val > G) { G = val; ep = k; eext = b > a; }
            }
            int Fv = NEG_INF, fext = 0;
            if (j - 1 >= lo[v]) {
                const int hv = h[t - 1], fv = f[t - 1];
                const int a = hv <= NEG_INF ? NEG_INF : hv - O - E;
                const int b = fv <= NEG_INF ? NEG_INF : fv - E;
                Fv = b > a ? b : a;
                fext = b > a;
            }
            int Hv = D, src = 0;
            if (G > Hv) { Hv = G; src = 1; }
            if (Fv > Hv) { Hv = Fv; src = 2; }
            if (Hv < NEG_INF) Hv = NEG_INF;
            if (D < NEG_INF) D = NEG_INF;
            h[t] = Hv; e[t] = G < NEG_INF ? NEG_INF : G; f[t] = Fv < NEG_INF ? NEG_INF : Fv;
            code[(size_t)v * W + t] = (uint16_t)(src | (eext << 2) | (fext << 3) | (dp << 4) | (ep << 10));
            if (Hv > best) { best = Hv; bj = j; }
        }
        mpos[v] = bj;
    }
    /* end: best pred of the sink at column m */
    int ub = -1, bs = NEG_INF;
    {
        const int32_t *pr = g->in_pred + (size_t)1 * POA_MAX_IN;
        for (int k = 0; k < g->nin[1]; k++) {
            const int u = pr[k];
            if (m < lo[u] || m > hi[u]) continue;
            const int hv = H[(size_t)u * W + (m - lo[u])];
            if (hv <= NEG_INF) continue;
            if (ub < 0 || hv > bs) { bs = hv; ub = u; }
        }
    }
    if (ub < 0) return -1;
    /* traceback (backward), then reverse */
    int n = 0, v = ub, j = m, state = 0;
    for (;;) {
        if (v == 0) {
            for (int jj = j; jj >= 1; jj--) path[n++] = (step_t){1, -1, jj - 1};
            break;
        }
        const uint16_t cd = code[(size_t)v * W + (j - lo[v])];
        if (state == 0) {
            const int src = cd & 3;
            if (src == 0) {
                path[n++] = (step_t){0, v, j - 1};
                v = g->in_pred[(size_t)v * POA_MAX_IN + ((cd >> 4) & 63)];
                j -= 1;
            } else {
                state = src;
            }
        } else if (state == 1) {
            path[n++] = (step_t){2, v, -1};
            const int u = g->in_pred[(size_t)v * POA_MAX_IN + ((cd >> 10) & 63)];
            state = (cd >> 2) & 1 ? 1 : 0;
            v = u;
        } else {
            path[n++] = (step_t){1, -1, j - 1};
            state = (cd >> 3) & 1 ? 2 : 0;
            j -= 1;
        }
    }
    for (int a = 0, b = n - 1; a < b; a++, b--) { step_t t = path[a]; path[a] = path[b]; path[b] = t; }
    return n;
}

/* The member of x's aligned group (x included) with the largest rank: the group's block end
 * (aligned groups are kept contiguous in the order). */
static int block_end(const graph_t *g, int x, const int32_t *rank) {
    int e = x;
    for (int q = 0; q < g->nal[x]; q++) {
        const int y = g->al[(size_t)x * POA_MAX_ALIGNED + q];
        if (rank[y] > rank[e]) e = y;
    }
    return e;
}

/* Fuse the aligned path into the graph and rebuild the topological order.  New nodes form
 * chains, each placed right after one existing node (its anchor) in path order: a mismatch
 * node starts a chain anchored at the end of its aligned group's block; an insertion node
 * extends the chain of the new node before it, or starts one anchored at the block end of
 * the existing node before it (the source for a leading insertion).  Aligned groups stay
 * contiguous and every new edge goes forward, so the order stays topological. */
static void fuse(graph_t *g, const uint8_t *s, const step_t *path, int n, int32_t *rank, int32_t *chain_head,
                 int32_t *chain_next, int32_t *chain_tail) {
    const int first_new = g->n;
    for (int r = 0; r < g->nord; r++) rank[g->ord[r]] = r;
    for (int i = 0; i < g->n; i++) chain_head[i] = -1;
    int prev = 0, cur = -1;   /* cur: anchor of the chain the previous new node belongs to */
    for (int k = 0; k < n; k++) {
        int x = -1, anchor = -1, is_new = 0;
        if (path[k].kind == 0) {
            const int v = path[k].node;
            const uint8_t b = s[path[k].j];
            if (g->base[v] == b) x = v;
            else {
                for (int q = 0; q < g->nal[v]; q++) {
                    const int y = g->al[(size_t)v * POA_MAX_ALIGNED + q];
                    if (g->base[y] == b) { x = y; break; }
                }
                if (x < 0) {
                    anchor = block_end(g, v, rank);   /* before x joins the group */
                    x = new_node(g, b);
                    join_group(g, v, x);
                    is_new = 1;
                }
            }
        } else if (path[k].kind == 1) {
            x = new_node(g, s[path[k].j]);
            anchor = prev >= first_new ? cur : (prev == 0 ? 0 : block_end(g, prev, rank));
            is_new = 1;
        }
        if (x < 0) continue;
        if (is_new) {
            chain_next[x] = -1;
            if (anchor == cur && prev >= first_new && path[k].kind == 1) {
                chain_next[chain_tail[anchor]] = x;   /* extends the current chain */
            } else {
                chain_head[anchor] = x;               /* one chain per anchor per path */
            }
            chain_tail[anchor] = x;
            cur = anchor;
        }
        add_edge(g, prev, x);
        prev = x;
    }
    add_edge(g, prev, 1);
    int no = 0;
    int32_t *nord = (int32_t *)malloc(sizeof(int32_t) * (size_t)g->n);
    for (int r = 0; r < g->nord; r++) {
        const int y = g->ord[r];
        nord[no++] = y;
        for (int x = chain_head[y]; x >= 0; x = chain_next[x]) nord[no++] = x;
    }
    memcpy(g->ord, nord, sizeof(int32_t) * (size_t)no);
    g->nord = no;
    free(nord);
}

int orc_poa_consensus(const uint8_t *bases, const uint64_t *off, int nseq, const orc_poa_params *pp,
                      uint8_t *out, int cap, int32_t *nused) {
    *nused = 0;
    if (nseq <= 0) return 0;
    const int maxn = pp->max_nodes;
    graph_t g;
    if (g_init(&g, maxn + 2)) { g_free(&g); return -1; }
    int maxm = 0;
    for (int i = 0; i < nseq; i++) {
        int m = (int)(off[i + 1] - off[i]);
        if (m > maxm) maxm = m;
    }
    const int W = 2 * (pp->band_b + (int)((int64_t)pp->band_f_permille * maxm / 1000)) + 2;
    int32_t *H = (int32_t *)malloc(sizeof(int32_t) * (size_t)(maxn + 2) * W);
    int32_t *Eg = (int32_t *)malloc(sizeof(int32_t) * (size_t)(maxn + 2) * W);
    int32_t *F = (int32_t *)malloc(sizeof(int32_t) * (size_t)(maxn + 2) * W);
    uint16_t *code = (uint16_t *)malloc(sizeof(uint16_t) * (size_t)(maxn + 2) * W);
    int32_t *lo = (int32_t *)malloc(sizeof(int32_t) * (size_t)(maxn + 2));
    int32_t *hi = (int32_t *)malloc(sizeof(int32_t) * (size_t)(maxn + 2));
    int32_t *mpos = (int32_t *)malloc(sizeof(int32_t) * (size_t)(maxn + 2));
    int32_t *rank = (int32_t *)malloc(sizeof(int32_t) * (size_t)(maxn + 2));
    int32_t *tmp = (int32_t *)malloc(sizeof(int32_t) * (size_t)(2 * maxn + 2 * maxm + 8));
    int32_t *rb = (int32_t *)malloc(sizeof(int32_t) * (size_t)(maxn + 2));
    int32_t *rl = (int32_t *)malloc(sizeof(int32_t) * (size_t)(maxn + 2));
    step_t *path = (step_t *)malloc(sizeof(step_t) * (size_t)(maxn + maxm + 8));
    int len = -1;
    if (!H || !Eg || !F || !code || !lo || !hi || !mpos || !rank || !tmp || !rb || !rl || !path) goto done;
    int used = 0;
    for (int i = 0; i < nseq && used < pp->max_seqs; i++) {
        const uint8_t *s = bases + off[i];
        const int m = (int)(off[i + 1] - off[i]);
        if (m < 1 || g.n - 2 + m > maxn) continue;
        if (g.n == 2) {   /* first sequence: a chain */
            int prev = 0;
            g.ord[0] = 0;
            for (int k = 0; k < m; k++) {
                const int x = new_node(&g, s[k]);
                add_edge(&g, prev, x);
                prev = x;
                g.ord[k + 1] = x;
            }
            add_edge(&g, prev, 1);
            g.ord[m + 1] = 1;
            g.nord = m + 2;
            used++;
            continue;
        }
        const int n = align(&g, s, m, pp, path, H, Eg, F, code, lo, hi, mpos, rank, W);
        if (n < 0) continue;
        fuse(&g, s, path, n, rank, rb, rl, tmp);
        used++;
    }
    *nused = used;
    /* heaviest bundle */
    {
        int32_t *score = mpos, *bp = rank;   /* reuse */
        score[0] = 0;
        bp[0] = -1;
        for (int r = 1; r < g.nord; r++) {
            const int v = g.ord[r];
            int bw = -1, bsc = 0, bu = -1;
            for (int k = 0; k < g.nin[v]; k++) {
                const int u = g.in_pred[(size_t)v * POA_MAX_IN + k], wt = g.in_w[(size_t)v * POA_MAX_IN + k];
                if (bu < 0 || wt > bw || (wt == bw && score[u] > bsc)) { bw = wt; bsc = score[u]; bu = u; }
            }
            bp[v] = bu;
            score[v] = bu < 0 ? 0 : bw + bsc;
        }
        int n = 0;
        for (int v = bp[1]; v >= 2; v = bp[v]) tmp[n++] = g.base[v];   /* node ids >= 2 carry bases */
        for (int k = 0; k < n && k < cap; k++) out[k] = (uint8_t)tmp[n - 1 - k];
        len = n;   /* the true length, even when > cap */
    }
done:
    free(H); free(Eg); free(F); free(code); free(lo); free(hi); free(mpos); free(rank); free(tmp); free(rb);
    free(rl); free(path);
    g_free(&g);
    return len;
}

/* ------------------------------------------------------------------ support selection */
/* The inserted sequences that support a refined INS call R: every I op with len >= 50
 * (refinement.c:299) of the reads refine_ins's region query yields for [s, e]
 * (refinement.c:290-293), processed by its walk (walk position before the op <= e,
 * refinement.c:305-316), with |position - R| <= support_radius and len <= max_len, in read
 * then op order.  ins_base[r] = index of read r's first such op (len >= 50) in the
 * pileup-wide (read, op) order of the insertion-sequence arrays. */
int orc_poa_support(const orc_pileup *p, const uint64_t *ins_base, int chrom, uint32_t s, uint32_t e,
                    uint32_t refined, const orc_poa_params *pp, int64_t *idx, int cap) {
    const int tid = chrom - 1;
    const int64_t beg = (int64_t)(uint32_t)(s - 1u), end = (int64_t)(uint32_t)(e - 1u);
    if (tid < 0 || tid >= p->n_targets || end <= beg) return 0;
    int n = 0;
    for (int64_t r = p->tid_off[tid]; r < p->tid_off[tid + 1]; r++) {
        if (!((int64_t)p->pos[r] < end && (int64_t)p->endpos[r] > beg)) continue;
        const uint32_t *cig = p->cigar + p->cig_off[r];
        const uint32_t nc = (uint32_t)(p->cig_off[r + 1] - p->cig_off[r]);
        uint32_t rp = (uint32_t)p->pos[r];
        uint64_t k = ins_base[r];
        for (uint32_t i = 0; i < nc; i++) {
            const uint32_t op = cig[i] & 0xfu, len = cig[i] >> 4;
            if (op == 1 && len >= 50) {
                const int64_t d = (int64_t)rp - (int64_t)refined;
                if ((d < 0 ? -d : d) <= pp->support_radius && (int)len <= pp->max_len) {
                    if (n < cap) idx[n] = (int64_t)k;
                    n++;
                }
                k++;
            }
            if (op != 1 && op != 4) rp += len;
            if (rp > e) break;
        }
    }
    return n;
}
