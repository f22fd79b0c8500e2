/*
 * simpileup.c -- seeded synthetic long-read pileups + BAM writer (see simpileup.h).
 *
 * Deterministic for a given sim_config (xoshiro256** PRNG, no libc rand), so tests on
 * this container and runs on the GPU box see identical inputs.  Output is columnar and
 * per-contig sorted by pos, exactly the svt_pileup_view layout (include/svtrek_gpu.h).
 */
#include "simpileup.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

enum { OP_M = 0, OP_I = 1, OP_D = 2, OP_N = 3, OP_S = 4, OP_H = 5, OP_P = 6, OP_EQ = 7, OP_X = 8 };

/* ---------------------------------------------------------------- PRNG */
typedef struct { uint64_t s[4]; } rng_t;
static uint64_t splitmix(uint64_t *x) {
    uint64_t z = (*x += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
static void rng_seed(rng_t *r, uint64_t seed) {
    for (int i = 0; i < 4; i++) r->s[i] = splitmix(&seed);
}
static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static inline uint64_t rng_u64(rng_t *r) {
    uint64_t *s = r->s, res = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return res;
}
static inline double rng_unif(rng_t *r) { return (double)(rng_u64(r) >> 11) * (1.0 / 9007199254740992.0); }
static inline int32_t rng_int(rng_t *r, int32_t lo, int32_t hi) {   /* inclusive */
    return lo + (int32_t)(rng_u64(r) % (uint64_t)(hi - lo + 1));
}
static inline double rng_norm(rng_t *r) {
    double u1 = rng_unif(r), u2 = rng_unif(r);
    if (u1 < 1e-300) u1 = 1e-300;
    return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}
static inline int32_t rng_geom(rng_t *r, double mean) {
    double u = rng_unif(r);
    if (u < 1e-300) u = 1e-300;
    int32_t v = (int32_t)(-log(u) * mean) + 1;
    return v < 1 ? 1 : v;
}

/* ---------------------------------------------------------------- storage */
typedef struct { int32_t type, chrom, pos, end, bp1, bp2, tid; } locus_t;

struct sim_pileup {
    int32_t   n_targets;
    int32_t  *contig_len;
    int64_t   n_reads;
    uint64_t  n_ops;
    int64_t  *tid_off;
    int32_t  *pos, *endpos;
    uint64_t *cig_off;
    uint32_t *cigar;
    uint16_t *flag;
    int32_t   n_loci;
    int32_t  *loci;    /* type, chrom, pos, end */
    int32_t  *truth;   /* bp1, bp2 */
};

typedef struct {           /* unsorted read list while generating */
    int32_t  *pos;  uint16_t *flag; uint64_t *off; int32_t *tid;
    int64_t   n, cap;
    uint32_t *ops;  uint64_t nops, capops;
} rbuf;

static int rb_reserve_ops(rbuf *b, uint64_t extra) {
    if (b->nops + extra <= b->capops) return 0;
    uint64_t nc = b->capops ? b->capops : (1u << 20);
    while (nc < b->nops + extra) nc *= 2;
    uint32_t *x = (uint32_t *)realloc(b->ops, nc * sizeof(uint32_t));
    if (!x) return -1;
    b->ops = x; b->capops = nc;
    return 0;
}
static int rb_begin(rbuf *b, int32_t tid, int32_t pos, uint16_t flag) {
    if (b->n == b->cap) {
        int64_t nc = b->cap ? b->cap * 2 : 4096;
        int32_t *p = (int32_t *)realloc(b->pos, (size_t)nc * sizeof(int32_t));
        if (!p) return -1;
        b->pos = p;
        uint16_t *f = (uint16_t *)realloc(b->flag, (size_t)nc * sizeof(uint16_t));
        if (!f) return -1;
        b->flag = f;
        uint64_t *o = (uint64_t *)realloc(b->off, (size_t)(nc + 1) * sizeof(uint64_t));
        if (!o) return -1;
        b->off = o;
        int32_t *t = (int32_t *)realloc(b->tid, (size_t)nc * sizeof(int32_t));
        if (!t) return -1;
        b->tid = t;
        b->cap = nc;
    }
    b->pos[b->n] = pos; b->flag[b->n] = flag; b->tid[b->n] = tid; b->off[b->n] = b->nops;
    return 0;
}
static inline void rb_op(rbuf *b, uint32_t op, uint32_t len) {
    if (len == 0) return;
    /* merge with the previous op of the same read when identical (keeps CIGARs canonical) */
    if (b->nops > b->off[b->n] && (b->ops[b->nops - 1] & 0xf) == op && op != OP_S && op != OP_H) {
        b->ops[b->nops - 1] += len << 4;
        return;
    }
    b->ops[b->nops++] = (len << 4) | op;
}
static inline void rb_end(rbuf *b) { b->n++; b->off[b->n] = b->nops; }

/* ---------------------------------------------------------------- read model */
typedef struct {
    const sim_config *c;
    rng_t *r;
    rbuf *b;
    const locus_t *sv; int32_t nsv;   /* SVs of this contig sorted by bp1 */
    int32_t tid, clen;
} gen_t;

static void small_event(gen_t *g, int32_t *ref, int32_t *q) {
    rng_t *r = g->r;
    double u = rng_unif(r);
    if (g->c->p_exotic > 0 && rng_unif(r) < g->c->p_exotic) {
        int32_t k = rng_int(r, 0, 5);
        uint32_t op = k == 0 ? OP_N : k == 1 ? OP_H : k == 2 ? OP_P : (uint32_t)rng_int(r, 9, 15);
        int32_t len = rng_int(r, 1, 60);
        rb_op(g->b, op, (uint32_t)len);
        /* the reference walk advances rp on every op but I and S (refinement.c:141) */
        *ref += len;
        return;
    }
    int32_t len = rng_int(r, 1, 5);
    if (u < 0.40) { rb_op(g->b, OP_X, (uint32_t)len); *ref += len; *q -= len; }
    else if (u < 0.70) { rb_op(g->b, OP_I, (uint32_t)len); *q -= len; }
    else { rb_op(g->b, OP_D, (uint32_t)len); *ref += len; }
}

/* Build one read starting at `start`, query length `qlen`.  Emits the primary (and a
 * supplementary for split reads).  Returns 0 / -1 on OOM. */
static int make_read(gen_t *g, int32_t start, int32_t qlen, int32_t *sv_cursor) {
    const sim_config *c = g->c;
    rng_t *r = g->r;
    rbuf *b = g->b;
    if (rb_reserve_ops(b, 3ull * (uint64_t)qlen + 16)) return -1;   /* <= 3 ops per loop turn, >= 1 base each */
    if (rb_begin(b, g->tid, start, 0)) return -1;
    int32_t ref = start, q = qlen;
    /* leading clip */
    if (rng_unif(r) < c->p_clip_ends) {
        int32_t k = rng_int(r, 1, 200);
        rb_op(b, rng_unif(r) < 0.8 ? OP_S : OP_H, (uint32_t)k);
    }
    int noise_done = rng_unif(r) >= c->p_noise_sv;
    int32_t cur = *sv_cursor;
    while (cur < g->nsv && g->sv[cur].bp1 < start) cur++;   /* first SV at/after read start */
    double mean_m = c->rho > 0 ? 2.0 / c->rho : 1e9;   /* each error event = M + op: rho ops/bp */
    int split = 0;
    int32_t split_ref = 0, split_q = 0;
    while (q > 0 && ref < g->clen - 1) {
        int32_t m = rng_geom(r, mean_m);
        if (m > q) m = q;
        if (cur < g->nsv && ref + m >= g->sv[cur].bp1) {
            const locus_t *sv = &g->sv[cur];
            int32_t j1 = c->bp_jitter ? rng_int(r, -c->bp_jitter, c->bp_jitter) : 0;
            int32_t bp1 = sv->bp1 + j1;
            if (bp1 <= ref) bp1 = ref + 1;
            int32_t mm = bp1 - ref;
            if (mm > q) { rb_op(b, OP_M, (uint32_t)q); ref += q; q = 0; break; }
            rb_op(b, OP_M, (uint32_t)mm); ref += mm; q -= mm;
            cur++;
            double u = rng_unif(r);
            if (sv->type == 2) {           /* DEL */
                int32_t j2 = c->bp_jitter ? rng_int(r, -c->bp_jitter, c->bp_jitter) : 0;
                int32_t dl = sv->bp2 + j2 - bp1;
                if (dl < 1) dl = 1;
                if (u < c->p_split) {
                    split = 1; split_ref = ref + dl; split_q = q;
                    rb_op(b, OP_S, (uint32_t)(q > 0 ? q : 1));
                    q = 0;
                    break;
                } else if (u < c->p_split + c->p_carry) {
                    rb_op(b, OP_D, (uint32_t)dl); ref += dl;
                }
            } else {                       /* INS */
                int32_t il = sv->bp2 - sv->bp1;
                if (il < 1) il = 1;
                if (u < c->p_carry) { rb_op(b, OP_I, (uint32_t)il); q -= il < q ? il : q; }
            }
            continue;
        }
        rb_op(b, OP_M, (uint32_t)m); ref += m; q -= m;
        if (q <= 0) break;
        if (!noise_done && rng_unif(r) < 0.01) {
            noise_done = 1;
            int32_t len = rng_int(r, 45, 400);
            if (rng_unif(r) < 0.5) { rb_op(b, OP_D, (uint32_t)len); ref += len; }
            else { rb_op(b, OP_I, (uint32_t)len); q -= len; }
            continue;
        }
        small_event(g, &ref, &q);
    }
    if (!split && rng_unif(r) < c->p_clip_ends) {
        int32_t k = rng_int(r, 1, 200);
        rb_op(b, rng_unif(r) < 0.8 ? OP_S : OP_H, (uint32_t)k);
    }
    if (b->nops == b->off[b->n]) rb_op(b, OP_M, 1);   /* never emit n_cigar == 0 */
    rb_end(b);
    if (split && split_ref < g->clen - 1 && split_q > 0) {
        /* supplementary: leading H (or S) for the clipped prefix, then the rest aligned */
        if (rb_reserve_ops(b, 3ull * (uint64_t)split_q + 16)) return -1;
        if (rb_begin(b, g->tid, split_ref, 0x800)) return -1;
        rb_op(b, rng_unif(r) < 0.5 ? OP_H : OP_S, (uint32_t)(qlen - split_q > 0 ? qlen - split_q : 1));
        int32_t ref2 = split_ref, q2 = split_q;
        while (q2 > 0 && ref2 < g->clen - 1) {
            int32_t m = rng_geom(r, mean_m);
            if (m > q2) m = q2;
            rb_op(b, OP_M, (uint32_t)m); ref2 += m; q2 -= m;
            if (q2 <= 0) break;
            small_event(g, &ref2, &q2);
        }
        if (b->nops == b->off[b->n] + 1) rb_op(b, OP_M, 1);
        rb_end(b);
    }
    return 0;
}

/* htslib bam_endpos: pos + (unmapped ? 0 : sum of M/D/N/=/X lengths), 0 -> 1 */
static int32_t endpos_of(int32_t pos, uint16_t flag, const uint32_t *ops, uint64_t n) {
    int64_t rl = 0;
    if (!(flag & 4))
        for (uint64_t i = 0; i < n; i++) {
            uint32_t op = ops[i] & 0xf;
            if (op == OP_M || op == OP_D || op == OP_N || op == OP_EQ || op == OP_X) rl += ops[i] >> 4;
        }
    if (rl == 0) rl = 1;
    return (int32_t)(pos + rl);
}

static int cmp_locus(const void *a, const void *b) {
    const locus_t *x = (const locus_t *)a, *y = (const locus_t *)b;
    return (x->bp1 > y->bp1) - (x->bp1 < y->bp1);
}

typedef struct { int32_t pos; int32_t idx; } sortkey_t;
static int cmp_key(const void *a, const void *b) {
    const sortkey_t *x = (const sortkey_t *)a, *y = (const sortkey_t *)b;
    if (x->pos != y->pos) return (x->pos > y->pos) - (x->pos < y->pos);
    return (x->idx > y->idx) - (x->idx < y->idx);
}


/* Reads of contig t (its SVs sv[0..nsv), sorted by bp1) whose start lies before x_end,
 * starting from x0, appended to b. 0 / -1 on OOM. */
static int gen_contig(const sim_config *c, rng_t *rng, rbuf *b, const locus_t *sv, int32_t nsv, int32_t t, int32_t clen,
                      double x0, double x_end) {
    gen_t g = {c, rng, b, sv, nsv, t, clen};
    int32_t cursor = 0;
    double mean_gap = (double)c->read_len_mean / (c->coverage > 0 ? c->coverage : 1.0);
    double x = x0;
    for (;;) {
        double u = rng_unif(rng);
        if (u < 1e-300) u = 1e-300;
        x += -log(u) * mean_gap;
        if (x >= x_end) break;
        int32_t qlen = (int32_t)(c->read_len_mean + c->read_len_sd * rng_norm(rng));
        if (qlen < c->read_len_min) qlen = c->read_len_min;
        int32_t start = (int32_t)x;
        if (start < 0) { qlen += start; start = 0; if (qlen < 1) continue; }
        while (cursor < g.nsv && g.sv[cursor].bp2 + 2 * c->bp_jitter + 2 < start) cursor++;
        if (make_read(&g, start, qlen, &cursor)) return -1;
    }
    return 0;
}

static void rb_free(rbuf *b) { free(b->pos); free(b->flag); free(b->off); free(b->tid); free(b->ops); memset(b, 0, sizeof *b); }

/* The reads of one contig -- reads [r0[q], r1[q]) of the buffers b[q], q < nb, in generation
 * order -- sorted by pos (ties: generation order) into p's arrays from read w / op wo on. */
static int emit_contig(sim_pileup *p, const rbuf *const *b, const int64_t *r0, const int64_t *r1, int nb, int64_t w,
                       uint64_t wo) {
    int64_t k = 0;
    for (int q = 0; q < nb; q++) k += r1[q] - r0[q];
    if (k > INT32_MAX) return -1;
    sortkey_t *keys = (sortkey_t *)malloc((size_t)(k > 0 ? k : 1) * sizeof(sortkey_t));
    int32_t *src = (int32_t *)malloc((size_t)(k > 0 ? k : 1) * sizeof(int32_t));   /* buffer of key i */
    if (!keys || !src) { free(keys); free(src); return -1; }
    int64_t i = 0;
    for (int q = 0; q < nb; q++)
        for (int64_t r = r0[q]; r < r1[q]; r++, i++) { keys[i].pos = b[q]->pos[r]; keys[i].idx = (int32_t)i; src[i] = q; }
    qsort(keys, (size_t)k, sizeof(sortkey_t), cmp_key);
    int64_t *base = (int64_t *)malloc(sizeof(int64_t) * (size_t)(nb + 1));
    if (!base) { free(keys); free(src); return -1; }
    base[0] = 0;
    for (int q = 0; q < nb; q++) base[q + 1] = base[q] + (r1[q] - r0[q]);
    for (int64_t j = 0; j < k; j++) {
        const int q = src[keys[j].idx];
        const rbuf *bb = b[q];
        const int64_t s = r0[q] + (keys[j].idx - base[q]);
        uint64_t n = bb->off[s + 1] - bb->off[s];
        memcpy(p->cigar + wo, bb->ops + bb->off[s], n * sizeof(uint32_t));
        p->pos[w] = bb->pos[s];
        p->flag[w] = bb->flag[s];
        p->cig_off[w] = wo;
        p->endpos[w] = endpos_of(bb->pos[s], bb->flag[s], p->cigar + wo, n);
        wo += n;
        w++;
    }
    free(keys); free(src); free(base);
    return 0;
}

static int alloc_reads(sim_pileup *p, int64_t nr, uint64_t nops, int32_t nt) {
    p->n_reads = nr;
    p->n_ops = nops;
    p->tid_off = (int64_t *)calloc((size_t)nt + 1, sizeof(int64_t));
    p->pos = (int32_t *)malloc((size_t)(nr > 0 ? nr : 1) * sizeof(int32_t));
    p->endpos = (int32_t *)malloc((size_t)(nr > 0 ? nr : 1) * sizeof(int32_t));
    p->flag = (uint16_t *)malloc((size_t)(nr > 0 ? nr : 1) * sizeof(uint16_t));
    p->cig_off = (uint64_t *)malloc((size_t)(nr + 1) * sizeof(uint64_t));
    p->cigar = (uint32_t *)malloc((size_t)(nops > 0 ? nops : 1) * sizeof(uint32_t));
    return p->tid_off && p->pos && p->endpos && p->flag && p->cig_off && p->cigar;
}

/* One PRNG stream for loci and then every contig in order (configs 1-4: the data of rounds 1-2). */
static int gen_serial(const sim_config *c, sim_pileup *p, locus_t *L, int32_t per, rng_t *rng) {
    rbuf b;
    memset(&b, 0, sizeof b);
    b.off = (uint64_t *)calloc(1, sizeof(uint64_t));
    if (!b.off) return 0;
    for (int32_t t = 0; t < c->n_targets; t++) {
        int32_t n0 = t * per, n1 = (t + 1) * per;
        if (n1 > c->n_loci) n1 = c->n_loci;
        if (n0 > n1) n0 = n1;
        qsort(L + n0, (size_t)(n1 - n0), sizeof(locus_t), cmp_locus);
        /* starts drift in from before 0 */
        if (gen_contig(c, rng, &b, L + n0, n1 - n0, t, p->contig_len[t], -(double)c->read_len_mean,
                       (double)(p->contig_len[t] - 1))) { rb_free(&b); return 0; }
    }
    if (!alloc_reads(p, b.n, b.nops, c->n_targets)) { rb_free(&b); return 0; }
    int64_t w = 0, r0 = 0;
    uint64_t wo = 0;
    for (int32_t t = 0; t < c->n_targets; t++) {   /* supplementaries were appended out of order */
        int64_t r1 = r0;
        while (r1 < b.n && b.tid[r1] == t) r1++;
        p->tid_off[t] = w;
        const rbuf *bp = &b;
        if (emit_contig(p, &bp, &r0, &r1, 1, w, wo)) { rb_free(&b); return 0; }
        wo += b.off[r1] - b.off[r0];
        w += r1 - r0;
        r0 = r1;
    }
    p->tid_off[c->n_targets] = w;
    p->cig_off[w] = wo;
    rb_free(&b);
    return 1;
}

/* par_contigs = K > 0: every contig in K segments of read starts, each from its own PRNG
 * stream (seeded from seed, contig and segment), one thread per segment -- configs too large
 * to generate serially (cfg5: 9 G CIGAR ops).  A different pileup than K = 0, equally seeded. */
typedef struct {
    const sim_config *c;
    sim_pileup *p;
    const locus_t *sv;
    int32_t nsv, t, k, K;
    rbuf b;
    int err;
} seg_job;

typedef struct {
    sim_pileup *p;
    seg_job *seg;   /* the contig's K segments */
    int32_t K;
    int64_t w;
    uint64_t wo;
    int err;
} emit_job_t;

static void *seg_run(void *arg) {
    seg_job *j = (seg_job *)arg;
    rng_t r;
    rng_seed(&r, j->c->seed ^ (0x9e3779b97f4a7c15ull * (uint64_t)(j->t + 1)) ^ (0xbf58476d1ce4e5b9ull * (uint64_t)j->k));
    const double clen = (double)(j->p->contig_len[j->t] - 1);
    const double x0 = j->k == 0 ? -(double)j->c->read_len_mean : clen * j->k / j->K;
    const double x1 = j->k + 1 == j->K ? clen : clen * (j->k + 1) / j->K;
    j->b.off = (uint64_t *)calloc(1, sizeof(uint64_t));
    j->err = !j->b.off || gen_contig(j->c, &r, &j->b, j->sv, j->nsv, j->t, j->p->contig_len[j->t], x0, x1);
    return NULL;
}

static void *emit_run(void *arg) {
    emit_job_t *j = (emit_job_t *)arg;
    const rbuf *bs[64];
    int64_t r0[64], r1[64];
    for (int32_t q = 0; q < j->K; q++) { bs[q] = &j->seg[q].b; r0[q] = 0; r1[q] = j->seg[q].b.n; }
    j->err = emit_contig(j->p, bs, r0, r1, j->K, j->w, j->wo) != 0;
    for (int32_t q = 0; q < j->K; q++) rb_free(&j->seg[q].b);
    return NULL;
}

static void run_all(void *(*fn)(void *), void *jobs, size_t size, int64_t n) {
    pthread_t *th = (pthread_t *)calloc((size_t)(n > 0 ? n : 1), sizeof(pthread_t));
    char *created = (char *)calloc((size_t)(n > 0 ? n : 1), 1);
    for (int64_t i = 0; i < n; i++) {
        void *a = (char *)jobs + (size_t)i * size;
        if (th && created && pthread_create(&th[i], NULL, fn, a) == 0) created[i] = 1;
        else fn(a);
    }
    for (int64_t i = 0; i < n; i++)
        if (created && created[i]) pthread_join(th[i], NULL);
    free(th);
    free(created);
}

static int gen_parallel(const sim_config *c, sim_pileup *p, locus_t *L, int32_t per) {
    const int32_t nt = c->n_targets, K = c->par_contigs > 64 ? 64 : c->par_contigs;
    seg_job *S = (seg_job *)calloc((size_t)nt * (size_t)K, sizeof(seg_job));
    emit_job_t *E = (emit_job_t *)calloc((size_t)nt, sizeof(emit_job_t));
    if (!S || !E) { free(S); free(E); return 0; }
    for (int32_t t = 0; t < nt; t++) {
        int32_t n0 = t * per, n1 = (t + 1) * per;
        if (n1 > c->n_loci) n1 = c->n_loci;
        if (n0 > n1) n0 = n1;
        qsort(L + n0, (size_t)(n1 - n0), sizeof(locus_t), cmp_locus);
        for (int32_t k = 0; k < K; k++) S[t * K + k] = (seg_job){c, p, L + n0, n1 - n0, t, k, K, {0}, 0};
    }
    run_all(seg_run, S, sizeof(seg_job), (int64_t)nt * K);
    int ok = 1;
    int64_t nr = 0;
    uint64_t nops = 0;
    for (int32_t t = 0; t < nt; t++) {
        E[t] = (emit_job_t){p, S + (size_t)t * K, K, nr, nops, 0};
        for (int32_t k = 0; k < K; k++) {
            ok &= !S[t * K + k].err;
            nr += S[t * K + k].b.n;
            nops += S[t * K + k].b.nops;
        }
    }
    if (ok) ok = alloc_reads(p, nr, nops, nt);
    if (ok) {
        for (int32_t t = 0; t < nt; t++) p->tid_off[t] = E[t].w;
        p->tid_off[nt] = nr;
        p->cig_off[nr] = nops;
        run_all(emit_run, E, sizeof(emit_job_t), nt);
        for (int32_t t = 0; t < nt; t++) ok &= !E[t].err;
    }
    for (int64_t i = 0; i < (int64_t)nt * K; i++) rb_free(&S[i].b);
    free(S);
    free(E);
    return ok;
}

sim_pileup *sim_generate(const sim_config *c) {
    if (!c || c->n_targets < 1 || c->n_loci < 0) return NULL;
    sim_pileup *p = (sim_pileup *)calloc(1, sizeof(sim_pileup));
    if (!p) return NULL;
    rng_t rng;
    rng_seed(&rng, c->seed);
    p->n_targets = c->n_targets;
    p->n_loci = c->n_loci;
    p->contig_len = (int32_t *)calloc((size_t)c->n_targets, sizeof(int32_t));
    p->loci = (int32_t *)calloc((size_t)(c->n_loci > 0 ? c->n_loci : 1) * 4, sizeof(int32_t));
    p->truth = (int32_t *)calloc((size_t)(c->n_loci > 0 ? c->n_loci : 1) * 2, sizeof(int32_t));
    locus_t *L = (locus_t *)calloc((size_t)(c->n_loci > 0 ? c->n_loci : 1), sizeof(locus_t));
    if (!p->contig_len || !p->loci || !p->truth || !L) { free(L); sim_free(p); return NULL; }

    /* loci: contig-major, evenly spaced with random offsets */
    int32_t per = (c->n_loci + c->n_targets - 1) / c->n_targets;
    if (per < 1) per = 1;
    for (int32_t t = 0; t < c->n_targets; t++)
        p->contig_len[t] = c->first_offset + per * c->spacing + c->first_offset;
    double lmin = log((double)c->sv_min_len), lmax = log((double)c->sv_max_len);
    for (int32_t k = 0; k < c->n_loci; k++) {
        int32_t t = k / per, slot = k % per;
        int32_t base = c->first_offset + slot * c->spacing;
        int32_t bp1 = base + rng_int(&rng, 0, c->spacing / 8);
        int32_t len = (int32_t)floor(exp(lmin + (lmax - lmin) * rng_unif(&rng)));
        if (len < c->sv_min_len) len = c->sv_min_len;
        int32_t type = rng_unif(&rng) < c->del_frac ? 2 : 1;
        int32_t bp2 = bp1 + len;
        int32_t rj = c->report_jitter;
        int32_t rpos = bp1 + (rj ? rng_int(&rng, -rj, rj) : 0);
        int32_t rend = type == 2 ? bp2 + (rj ? rng_int(&rng, -rj, rj) : 0) : rpos + 1;
        L[k] = (locus_t){type, t + 1, rpos, rend, bp1, bp2, t};
        p->loci[4 * k + 0] = type; p->loci[4 * k + 1] = t + 1;
        p->loci[4 * k + 2] = rpos; p->loci[4 * k + 3] = rend;
        p->truth[2 * k + 0] = bp1; p->truth[2 * k + 1] = bp2;
    }

    int ok = c->par_contigs ? gen_parallel(c, p, L, per) : gen_serial(c, p, L, per, &rng);
    free(L);
    if (!ok) { sim_free(p); return NULL; }
    return p;
}

void sim_free(sim_pileup *p) {
    if (!p) return;
    free(p->contig_len); free(p->tid_off); free(p->pos); free(p->endpos); free(p->cig_off);
    free(p->cigar); free(p->flag); free(p->loci); free(p->truth); free(p);
}

int32_t sim_n_targets(const sim_pileup *p) { return p->n_targets; }
int32_t sim_contig_len(const sim_pileup *p, int32_t t) { return (t >= 0 && t < p->n_targets) ? p->contig_len[t] : 0; }
int64_t sim_n_reads(const sim_pileup *p) { return p->n_reads; }
uint64_t sim_n_ops(const sim_pileup *p) { return p->n_ops; }
const int64_t *sim_tid_off(const sim_pileup *p) { return p->tid_off; }
const int32_t *sim_pos(const sim_pileup *p) { return p->pos; }
const int32_t *sim_endpos(const sim_pileup *p) { return p->endpos; }
const uint64_t *sim_cig_off(const sim_pileup *p) { return p->cig_off; }
const uint32_t *sim_cigar(const sim_pileup *p) { return p->cigar; }
const uint16_t *sim_flag(const sim_pileup *p) { return p->flag; }
int32_t sim_n_loci(const sim_pileup *p) { return p->n_loci; }
const int32_t *sim_loci(const sim_pileup *p) { return p->loci; }
const int32_t *sim_truth(const sim_pileup *p) { return p->truth; }

/* ---------------------------------------------------------------- insertion sequences */
typedef struct { int32_t bp1, len, k; } ins_key;

static int cmp_ins(const void *a, const void *b) {
    const ins_key *x = (const ins_key *)a, *y = (const ins_key *)b;
    return x->bp1 < y->bp1 ? -1 : x->bp1 > y->bp1 ? 1 : (x->k < y->k ? -1 : x->k > y->k);
}

void sim_free_buf(void *x) { free(x); }

int sim_insseq(const sim_pileup *p, uint64_t seed, int32_t bp_jitter, int32_t err_permille, uint64_t *n_ins,
               uint64_t **off_out, uint8_t **bases_out) {
    *n_ins = 0; *off_out = NULL; *bases_out = NULL;
    /* INS loci per contig, sorted by true bp1 */
    int32_t nt = p->n_targets;
    ins_key *keys = (ins_key *)malloc(sizeof(ins_key) * (size_t)(p->n_loci > 0 ? p->n_loci : 1));
    int64_t *koff = (int64_t *)calloc((size_t)nt + 1, sizeof(int64_t));
    if (!keys || !koff) { free(keys); free(koff); return -1; }
    int64_t nk = 0;
    for (int32_t t = 0; t < nt; t++) {
        koff[t] = nk;
        for (int32_t k = 0; k < p->n_loci; k++)
            if (p->loci[4 * k] == 1 && p->loci[4 * k + 1] == t + 1)
                keys[nk++] = (ins_key){p->truth[2 * k], p->truth[2 * k + 1] - p->truth[2 * k], k};
        qsort(keys + koff[t], (size_t)(nk - koff[t]), sizeof(ins_key), cmp_ins);
    }
    koff[nt] = nk;
    /* pass 1: sizes */
    uint64_t n = 0, nb = 0;
    for (int64_t r = 0; r < p->n_reads; r++)
        for (uint64_t i = p->cig_off[r]; i < p->cig_off[r + 1]; i++)
            if ((p->cigar[i] & 0xfu) == OP_I && (p->cigar[i] >> 4) >= 50) { n++; nb += p->cigar[i] >> 4; }
    uint64_t *off = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(n + 1));
    uint8_t *bases = (uint8_t *)malloc((size_t)(nb > 0 ? nb : 1));
    if (!off || !bases) { free(off); free(bases); free(keys); free(koff); return -1; }
    /* pass 2 */
    uint64_t q = 0, o = 0;
    rng_t rng;
    rng_seed(&rng, seed ^ 0x9e3779b97f4a7c15ull);
    for (int32_t t = 0; t < nt; t++) {
        for (int64_t r = p->tid_off[t]; r < p->tid_off[t + 1]; r++) {
            uint32_t rp = (uint32_t)p->pos[r];
            for (uint64_t i = p->cig_off[r]; i < p->cig_off[r + 1]; i++) {
                const uint32_t op = p->cigar[i] & 0xfu, len = p->cigar[i] >> 4;
                if (op == OP_I && len >= 50) {
                    off[q++] = o;
                    /* the INS locus whose allele this op carries, if any */
                    int64_t lo = koff[t], hi = koff[t + 1];
                    while (lo < hi) { int64_t m = (lo + hi) / 2; if ((int64_t)keys[m].bp1 < (int64_t)rp - bp_jitter - 1) lo = m + 1; else hi = m; }
                    int32_t k = -1;
                    for (int64_t m = lo; m < koff[t + 1] && (int64_t)keys[m].bp1 <= (int64_t)rp + bp_jitter + 1; m++)
                        if (keys[m].len == (int32_t)len) { k = keys[m].k; break; }
                    if (k >= 0) {
                        rng_t al;   /* the locus's allele: a per-locus stream */
                        rng_seed(&al, seed * 1000003ull + (uint64_t)k);
                        for (uint32_t b = 0; b < len; b++) {
                            uint8_t base = (uint8_t)(rng_u64(&al) & 3);
                            if ((int32_t)(rng_u64(&rng) % 1000) < err_permille)
                                base = (uint8_t)((base + 1 + rng_u64(&rng) % 3) & 3);
                            bases[o + b] = base;
                        }
                    } else {
                        for (uint32_t b = 0; b < len; b++) bases[o + b] = (uint8_t)(rng_u64(&rng) & 3);
                    }
                    o += len;
                }
                if (op != OP_I && op != OP_S) rp += len;
            }
        }
    }
    off[n] = o;
    free(keys); free(koff);
    *n_ins = n; *off_out = off; *bases_out = bases;
    return 0;
}

/* ---------------------------------------------------------------- BAM writer */
/* BGZF blocks are independent deflate streams, so the writer fills a batch of blocks and
 * compresses them on several threads, then writes them in order.  Virtual offsets handed out
 * while writing are (block index << 16 | in-block offset); the BAI is built afterwards with
 * each block index mapped to its file offset. */
#define BGZF_BLK 65280
#define BGZF_BATCH 256
#define BGZF_THREADS 16
typedef struct {
    FILE *f;
    uint8_t *ubuf;        /* BGZF_BATCH blocks of BGZF_BLK bytes */
    uint8_t *cbuf;        /* BGZF_BATCH compressed blocks of <= 65536 bytes */
    uint32_t *ulen, *clen;
    size_t nb;            /* complete blocks in the batch */
    size_t n;             /* bytes in the open block */
    uint64_t blk;         /* blocks written before this batch */
    uint64_t coff;        /* compressed bytes written so far */
    uint64_t *boff;       /* file offset of every block written */
    size_t capboff;
    int level;
    int err;
} bgzf_w;

/* virtual offset of the next byte written: (block index << 16 | in-block offset) */
static uint64_t bgzf_voff(const bgzf_w *w) { return (w->blk + w->nb) << 16 | (uint64_t)w->n; }

static int bgzf_block(uint8_t *out, const uint8_t *in, uint32_t n, int level, uint32_t *bsize) {
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    if (deflateInit2(&zs, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY) != Z_OK) return -1;
    zs.next_in = (Bytef *)in; zs.avail_in = (uInt)n;
    zs.next_out = out + 18; zs.avail_out = (uInt)(65536 - 26);
    if (deflate(&zs, Z_FINISH) != Z_STREAM_END) { deflateEnd(&zs); return -1; }
    size_t cl = zs.total_out;
    deflateEnd(&zs);
    size_t bs = cl + 26;   /* whole block */
    static const uint8_t hdr[16] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 'B', 'C', 2, 0};
    memcpy(out, hdr, 16);
    out[16] = (uint8_t)((bs - 1) & 0xff);
    out[17] = (uint8_t)((bs - 1) >> 8);
    uint32_t crc = (uint32_t)crc32(crc32(0L, Z_NULL, 0), in, (uInt)n);
    uint8_t *t = out + 18 + cl;
    t[0] = crc & 0xff; t[1] = (crc >> 8) & 0xff; t[2] = (crc >> 16) & 0xff; t[3] = crc >> 24;
    t[4] = n & 0xff; t[5] = (n >> 8) & 0xff; t[6] = (n >> 16) & 0xff; t[7] = n >> 24;
    *bsize = (uint32_t)bs;
    return 0;
}

typedef struct { bgzf_w *w; size_t k0, nblk, step; int err; } bgzf_job;
static void *bgzf_job_run(void *arg) {
    bgzf_job *j = (bgzf_job *)arg;
    for (size_t k = j->k0; k < j->nblk; k += j->step)
        if (bgzf_block(j->w->cbuf + k * 65536, j->w->ubuf + k * BGZF_BLK, j->w->ulen[k], j->w->level, &j->w->clen[k]))
            j->err = 1;
    return NULL;
}

/* compress the batch's blocks (the open one too when `last`) and write them in order */
static void bgzf_flush_batch(bgzf_w *w, int last) {
    if (last && w->n) { w->ulen[w->nb++] = (uint32_t)w->n; w->n = 0; }
    const size_t nb = w->nb;
    if (w->err || nb == 0) { w->nb = 0; return; }
    const size_t T = nb < BGZF_THREADS ? nb : BGZF_THREADS;
    bgzf_job J[BGZF_THREADS];
    pthread_t th[BGZF_THREADS];
    int made[BGZF_THREADS] = {0};
    for (size_t t = 0; t < T; t++) {
        J[t] = (bgzf_job){w, t, nb, T, 0};
        made[t] = pthread_create(&th[t], NULL, bgzf_job_run, &J[t]) == 0;
        if (!made[t]) bgzf_job_run(&J[t]);
    }
    for (size_t t = 0; t < T; t++) {
        if (made[t]) pthread_join(th[t], NULL);
        if (J[t].err) w->err = 1;
    }
    if (w->blk + nb > w->capboff) {
        size_t nc = w->capboff ? 2 * w->capboff : 1024;
        while (nc < w->blk + nb) nc *= 2;
        uint64_t *x = (uint64_t *)realloc(w->boff, nc * sizeof(uint64_t));
        if (!x) { w->err = 1; return; }
        w->boff = x; w->capboff = nc;
    }
    for (size_t k = 0; k < nb && !w->err; k++) {
        w->boff[w->blk + k] = w->coff;
        if (fwrite(w->cbuf + k * 65536, 1, w->clen[k], w->f) != w->clen[k]) w->err = 1;
        w->coff += w->clen[k];
    }
    w->blk += nb;
    w->nb = 0;
}

static void bgzf_put(bgzf_w *w, const void *data, size_t len) {
    const uint8_t *d = (const uint8_t *)data;
    while (len) {
        size_t k = BGZF_BLK - w->n;
        if (k > len) k = len;
        memcpy(w->ubuf + w->nb * BGZF_BLK + w->n, d, k);
        w->n += k; d += k; len -= k;
        if (w->n == BGZF_BLK) {   /* block complete */
            w->ulen[w->nb++] = BGZF_BLK;
            w->n = 0;
            if (w->nb == BGZF_BATCH) bgzf_flush_batch(w, 0);
        }
    }
}

static bgzf_w *bgzf_open(const char *path, int level) {
    bgzf_w *w = (bgzf_w *)calloc(1, sizeof(bgzf_w));
    if (!w) return NULL;
    w->ubuf = (uint8_t *)malloc((size_t)BGZF_BATCH * BGZF_BLK);
    w->cbuf = (uint8_t *)malloc((size_t)BGZF_BATCH * 65536);
    w->ulen = (uint32_t *)calloc(BGZF_BATCH, sizeof(uint32_t));
    w->clen = (uint32_t *)calloc(BGZF_BATCH, sizeof(uint32_t));
    w->f = fopen(path, "wb");
    w->level = level < 0 ? 6 : level;
    if (!w->ubuf || !w->cbuf || !w->ulen || !w->clen || !w->f) {
        if (w->f) fclose(w->f);
        free(w->ubuf); free(w->cbuf); free(w->ulen); free(w->clen); free(w);
        return NULL;
    }
    return w;
}

/* file offset << 16 | in-block offset of a virtual offset handed out by bgzf_voff */
static uint64_t bgzf_real(const bgzf_w *w, uint64_t v) {
    const uint64_t b = v >> 16;
    const uint64_t c = b < w->blk ? w->boff[b] : w->coff;   /* past the last block: EOF marker */
    return c << 16 | (v & 0xffff);
}

static void bgzf_free(bgzf_w *w) {
    free(w->ubuf); free(w->cbuf); free(w->ulen); free(w->clen); free(w->boff); free(w);
}
static void put32(bgzf_w *w, int32_t v) { uint8_t b[4] = {(uint8_t)v, (uint8_t)(v >> 8), (uint8_t)(v >> 16), (uint8_t)(v >> 24)}; bgzf_put(w, b, 4); }

/* SAM spec reg2bin for [beg, end) */
static int reg2bin(int64_t beg, int64_t end) {
    --end;
    if (beg >> 14 == end >> 14) return (int)(((1 << 15) - 1) / 7 + (beg >> 14));
    if (beg >> 17 == end >> 17) return (int)(((1 << 12) - 1) / 7 + (beg >> 17));
    if (beg >> 20 == end >> 20) return (int)(((1 << 9) - 1) / 7 + (beg >> 20));
    if (beg >> 23 == end >> 23) return (int)(((1 << 6) - 1) / 7 + (beg >> 23));
    if (beg >> 26 == end >> 26) return (int)(((1 << 3) - 1) / 7 + (beg >> 26));
    return 0;
}

/* ---------------------------------------------------------------- BAI (SAM spec 5.2) */
typedef struct { uint64_t beg, end; } bai_chunk;
typedef struct { uint32_t bin; int32_t n, cap; bai_chunk *c; } bai_bin;
typedef struct {
    bai_bin *bins;        /* indexed by bin number (37450 per reference, allocated lazily) */
    uint32_t *used;       /* bin numbers in first-use order */
    int32_t n_used;
    uint64_t *ioff;       /* linear index: 16 kb windows */
    int32_t n_intv, cap_intv;
} bai_ref;

#define BAI_NBIN 37450

static int bai_add(bai_ref *r, uint32_t bin, uint64_t beg, uint64_t end, int64_t pos, int64_t endpos) {
    if (!r->bins) {
        r->bins = (bai_bin *)calloc(BAI_NBIN, sizeof(bai_bin));
        r->used = (uint32_t *)malloc(BAI_NBIN * sizeof(uint32_t));
        if (!r->bins || !r->used) return -1;
    }
    bai_bin *b = &r->bins[bin];
    if (b->n == 0 && b->cap == 0) r->used[r->n_used++] = bin;
    b->bin = bin;
    if (b->n && b->c[b->n - 1].end == beg) {
        b->c[b->n - 1].end = end;   /* adjacent records of one bin: one chunk */
    } else {
        if (b->n == b->cap) {
            int32_t nc = b->cap ? 2 * b->cap : 4;
            bai_chunk *x = (bai_chunk *)realloc(b->c, (size_t)nc * sizeof(bai_chunk));
            if (!x) return -1;
            b->c = x; b->cap = nc;
        }
        b->c[b->n++] = (bai_chunk){beg, end};
    }
    /* linear index: every 16 kb window the record overlaps keeps its smallest offset */
    int64_t w0 = pos >> 14, w1 = (endpos > pos ? endpos - 1 : pos) >> 14;
    if (w1 >= r->cap_intv) {
        int32_t nc = r->cap_intv ? r->cap_intv : 64;
        while (nc <= w1) nc *= 2;
        uint64_t *x = (uint64_t *)realloc(r->ioff, (size_t)nc * sizeof(uint64_t));
        if (!x) return -1;
        for (int32_t i = r->cap_intv; i < nc; i++) x[i] = UINT64_MAX;
        r->ioff = x; r->cap_intv = nc;
    }
    for (int64_t k = w0; k <= w1; k++)
        if (r->ioff[k] == UINT64_MAX) r->ioff[k] = beg;
    if (w1 + 1 > r->n_intv) r->n_intv = (int32_t)(w1 + 1);
    return 0;
}

static int bai_write(bai_ref *refs, int32_t n_ref, const char *path) {
    FILE *f = fopen(path, "wb");
    if (!f) return -1;
    int err = fwrite("BAI\1", 1, 4, f) != 4;
    err |= fwrite(&n_ref, 4, 1, f) != 1;
    for (int32_t t = 0; t < n_ref; t++) {
        bai_ref *r = &refs[t];
        err |= fwrite(&r->n_used, 4, 1, f) != 1;
        for (int32_t i = 0; i < r->n_used; i++) {
            bai_bin *b = &r->bins[r->used[i]];
            err |= fwrite(&b->bin, 4, 1, f) != 1;
            err |= fwrite(&b->n, 4, 1, f) != 1;
            err |= fwrite(b->c, sizeof(bai_chunk), (size_t)b->n, f) != (size_t)b->n;
        }
        /* empty windows take the next non-empty window's offset (windows are monotone in a
         * coordinate-sorted file, so a query starting in an empty window loses nothing) */
        uint64_t nxt = 0;
        for (int32_t k = r->n_intv - 1; k >= 0; k--) {
            if (r->ioff[k] == UINT64_MAX) r->ioff[k] = nxt;
            else nxt = r->ioff[k];
        }
        err |= fwrite(&r->n_intv, 4, 1, f) != 1;
        if (r->n_intv) err |= fwrite(r->ioff, 8, (size_t)r->n_intv, f) != (size_t)r->n_intv;
    }
    uint64_t n_no_coor = 0;
    err |= fwrite(&n_no_coor, 8, 1, f) != 1;
    if (fclose(f)) err = 1;
    return err ? -1 : 0;
}

static void bai_free(bai_ref *refs, int32_t n_ref) {
    if (!refs) return;
    for (int32_t t = 0; t < n_ref; t++) {
        if (refs[t].bins)
            for (int32_t i = 0; i < refs[t].n_used; i++) free(refs[t].bins[refs[t].used[i]].c);
        free(refs[t].bins); free(refs[t].used); free(refs[t].ioff);
    }
    free(refs);
}

int sim_write_bam(const sim_pileup *p, const char *path, int with_seq, int level) {
    return sim_write_bam_region(p, path, with_seq, level, -1, 0, 0, 0);
}

int sim_write_bam_region(const sim_pileup *p, const char *path, int with_seq, int level, int32_t rtid, int64_t rbeg,
                         int64_t rend, int write_bai) {
    return sim_write_bam_regions(p, path, with_seq, level, rtid >= 0 ? 1 : 0, &rtid, &rbeg, &rend, write_bai);
}

/* a record of contig t is written when it overlaps one of the regions of t (all records when
 * nreg == 0) */
static int in_regions(int nreg, const int32_t *rt, const int64_t *rb, const int64_t *re, int32_t t, int64_t pos,
                      int64_t endpos) {
    if (nreg == 0) return 1;
    for (int k = 0; k < nreg; k++)
        if (rt[k] == t && pos < re[k] && endpos > rb[k]) return 1;
    return 0;
}

int sim_write_bam_regions(const sim_pileup *p, const char *path, int with_seq, int level, int nreg, const int32_t *rtid,
                          const int64_t *rbeg, const int64_t *rend, int write_bai) {
    bgzf_w *w = bgzf_open(path, level);
    if (!w) return -1;
    bai_ref *bai = NULL;
    if (write_bai && !(bai = (bai_ref *)calloc((size_t)(p->n_targets > 0 ? p->n_targets : 1), sizeof(bai_ref)))) {
        fclose(w->f);
        bgzf_free(w);
        return -1;
    }
    /* BAI entries, with virtual offsets mapped to file offsets once every block is written */
    typedef struct { int32_t t; uint32_t bin; uint64_t vb, ve; int64_t pos, endpos; } pend_t;
    pend_t *pend = NULL;
    size_t npend = 0, cappend = 0;
    rng_t rng;
    rng_seed(&rng, 0x5eed5eedull);
    /* header */
    char text[4096];
    int tl = snprintf(text, sizeof text, "@HD\tVN:1.6\tSO:coordinate\n");
    bgzf_put(w, "BAM\1", 4);
    /* @SQ lines can exceed the buffer for many contigs; emit them piecewise */
    size_t sq_len = 0;
    for (int t = 0; t < p->n_targets; t++) {
        char line[128];
        sq_len += (size_t)snprintf(line, sizeof line, "@SQ\tSN:%d\tLN:%d\n", t + 1, p->contig_len[t]);
    }
    put32(w, (int32_t)((size_t)tl + sq_len));
    bgzf_put(w, text, (size_t)tl);
    for (int t = 0; t < p->n_targets; t++) {
        char line[128];
        int k = snprintf(line, sizeof line, "@SQ\tSN:%d\tLN:%d\n", t + 1, p->contig_len[t]);
        bgzf_put(w, line, (size_t)k);
    }
    put32(w, p->n_targets);
    for (int t = 0; t < p->n_targets; t++) {
        char name[32];
        int k = snprintf(name, sizeof name, "%d", t + 1);
        put32(w, k + 1);
        bgzf_put(w, name, (size_t)k + 1);
        put32(w, p->contig_len[t]);
    }
    /* records */
    uint8_t *rec = NULL;
    size_t rec_cap = 0;
    static const char nt16[] = "=ACMGRSVTWYHKDBN";
    for (int t = 0; t < p->n_targets; t++) {
        int any = nreg == 0;
        for (int k = 0; k < nreg; k++) any |= rtid[k] == t;
        if (!any) continue;
        for (int64_t r = p->tid_off[t]; r < p->tid_off[t + 1]; r++) {
            if (!in_regions(nreg, rtid, rbeg, rend, t, p->pos[r], p->endpos[r])) continue;
            const uint32_t *ops = p->cigar + p->cig_off[r];
            uint64_t n = p->cig_off[r + 1] - p->cig_off[r];
            int64_t qlen = 0, rlen = 0;
            for (uint64_t i = 0; i < n; i++) {
                uint32_t op = ops[i] & 0xf, l = ops[i] >> 4;
                if (op == OP_M || op == OP_I || op == OP_S || op == OP_EQ || op == OP_X) qlen += l;
                if (op == OP_M || op == OP_D || op == OP_N || op == OP_EQ || op == OP_X) rlen += l;
            }
            int32_t l_seq = with_seq ? (int32_t)qlen : 0;
            char qname[32];
            int lq = snprintf(qname, sizeof qname, "r%lld", (long long)r) + 1;
            int use_cg = n > 65535;
            uint32_t n_cig_field = use_cg ? 2u : (uint32_t)n;
            size_t need = 32 + (size_t)lq + 4 * (size_t)n_cig_field + (size_t)(l_seq + 1) / 2 + (size_t)l_seq +
                          (use_cg ? 8 + 4 * n : 0);
            if (need > rec_cap) {
                rec_cap = need * 2;
                uint8_t *x = (uint8_t *)realloc(rec, rec_cap);
                if (!x) { free(rec); free(pend); fclose(w->f); bgzf_free(w); bai_free(bai, p->n_targets); return -1; }
                rec = x;
            }
            uint8_t *q = rec + 4;
            int32_t hdr32[8];
            hdr32[0] = t;
            hdr32[1] = p->pos[r];
            hdr32[2] = (int32_t)((uint32_t)reg2bin(p->pos[r], p->endpos[r]) << 16 | (uint32_t)60 << 8 | (uint32_t)lq);
            hdr32[3] = (int32_t)((uint32_t)p->flag[r] << 16 | n_cig_field);
            hdr32[4] = l_seq;
            hdr32[5] = -1; hdr32[6] = -1; hdr32[7] = 0;
            memcpy(q, hdr32, 32); q += 32;
            memcpy(q, qname, (size_t)lq); q += lq;
            if (use_cg) {
                uint32_t fake[2] = {(uint32_t)l_seq << 4 | OP_S, (uint32_t)rlen << 4 | OP_N};
                memcpy(q, fake, 8); q += 8;
            } else {
                memcpy(q, ops, 4 * n); q += 4 * n;
            }
            for (int32_t i = 0; i < (l_seq + 1) / 2; i++) {
                uint8_t a = (uint8_t)(1u << (rng_u64(&rng) & 3)), c2 = (uint8_t)(1u << (rng_u64(&rng) & 3));
                (void)nt16;
                *q++ = (uint8_t)(a << 4 | c2);
            }
            for (int32_t i = 0; i < l_seq; i++) *q++ = (uint8_t)(10 + (rng_u64(&rng) % 30));
            if (use_cg) {
                q[0] = 'C'; q[1] = 'G'; q[2] = 'B'; q[3] = 'I';
                uint32_t cnt = (uint32_t)n;
                memcpy(q + 4, &cnt, 4);
                memcpy(q + 8, ops, 4 * n);
                q += 8 + 4 * n;
            }
            int32_t bs = (int32_t)(q - rec - 4);
            memcpy(rec, &bs, 4);
            const uint64_t vbeg = bgzf_voff(w);
            bgzf_put(w, rec, (size_t)(q - rec));
            if (bai) {
                if (npend == cappend) {
                    cappend = cappend ? 2 * cappend : 4096;
                    pend_t *x = (pend_t *)realloc(pend, cappend * sizeof(pend_t));
                    if (!x) { w->err = 1; break; }
                    pend = x;
                }
                pend[npend++] = (pend_t){t, (uint32_t)reg2bin(p->pos[r], p->endpos[r]), vbeg, bgzf_voff(w), p->pos[r],
                                         p->endpos[r]};
            }
        }
    }
    free(rec);
    bgzf_flush_batch(w, 1);
    static const uint8_t eof[28] = {31, 139, 8, 4, 0, 0, 0, 0, 0, 255, 6, 0, 66, 67, 2, 0, 27, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (!w->err && fwrite(eof, 1, 28, w->f) != 28) w->err = 1;
    int err = w->err;
    if (fclose(w->f)) err = 1;
    for (size_t k = 0; bai && !err && k < npend; k++)
        if (bai_add(&bai[pend[k].t], pend[k].bin, bgzf_real(w, pend[k].vb), bgzf_real(w, pend[k].ve), pend[k].pos,
                    pend[k].endpos)) err = 1;
    free(pend);
    bgzf_free(w);
    if (bai && !err) {
        size_t L = strlen(path);
        char *bp = (char *)malloc(L + 5);
        if (!bp) err = 1;
        else {
            memcpy(bp, path, L);
            memcpy(bp + L, ".bai", 5);
            if (bai_write(bai, p->n_targets, bp)) err = 1;
            free(bp);
        }
    }
    bai_free(bai, p->n_targets);
    return err ? -1 : 0;
}
