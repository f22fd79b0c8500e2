/*
 * bgzf_ref.c -- TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg), never shipped.
 *
 * The reference's CPU path in the shape SURVEY.md §8(d) prescribes for the baseline: T
 * worker threads, each with its own BAM file handle and its own copy of the BAI
 * (audit.c:269-272: hts_open + sam_hdr_read + sam_index_load per thread), and per region
 * query what htslib's sam_itr_queryi / sam_itr_next do without a block cache
 * (refinement.c:114-117): take the query's start offset from the BAI's 16 kb linear index,
 * read and inflate BGZF blocks from there (zlib raw inflate, CRC not checked), copy each
 * record into a bam1_t-like buffer (bam_read1 copies the whole variable-length part, SEQ
 * and QUAL included), restore a CG:B,I CIGAR as bam_read1 does (htslib bam_tag2cigar), and
 * stop at the first record past the query (tid != query tid or pos >= end); records with
 * bam_endpos > beg are yielded.  The CIGAR walks and the vote are the oracle's own
 * (orc_refine_locus_src, svtrek_oracle.c), so this leg's results equal orc_refine_batch's
 * on the same pileup -- tests/test_bgzf_baseline.py checks that.
 *
 * htslib also merges the binning index's chunks for the query; on a coordinate-sorted
 * file the linear-index start reaches the same records (a few more, all before the
 * window), so the inflated byte count here is a lower bound of htslib's.
 */
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <zlib.h>

#include "svtrek_oracle.h"

enum { OP_M = 0, OP_D = 2, OP_N = 3, OP_S = 4, OP_EQ = 7, OP_X = 8 };

static uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint16_t rd16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }

/* ---------------------------------------------------------------- BAI (linear index only) */
typedef struct {
    int32_t n_ref;
    int32_t *n_intv;
    uint64_t **ioff;
} bai_t;

static void bai_free(bai_t *b) {
    if (!b) return;
    for (int32_t i = 0; i < b->n_ref; i++) free(b->ioff[i]);
    free(b->ioff); free(b->n_intv); free(b);
}

static bai_t *bai_load(const char *bam_path) {
    size_t L = strlen(bam_path);
    char *p = (char *)malloc(L + 5);
    if (!p) return NULL;
    memcpy(p, bam_path, L); memcpy(p + L, ".bai", 5);
    FILE *f = fopen(p, "rb");
    free(p);
    if (!f) return NULL;
    bai_t *b = (bai_t *)calloc(1, sizeof(bai_t));
    char magic[4];
    int ok = b && fread(magic, 1, 4, f) == 4 && memcmp(magic, "BAI\1", 4) == 0 && fread(&b->n_ref, 4, 1, f) == 1 &&
             b->n_ref >= 0;
    if (ok) {
        b->n_intv = (int32_t *)calloc((size_t)b->n_ref + 1, sizeof(int32_t));
        b->ioff = (uint64_t **)calloc((size_t)b->n_ref + 1, sizeof(uint64_t *));
        ok = b->n_intv && b->ioff;
    }
    for (int32_t r = 0; ok && r < b->n_ref; r++) {
        int32_t n_bin;
        ok = fread(&n_bin, 4, 1, f) == 1 && n_bin >= 0;
        for (int32_t i = 0; ok && i < n_bin; i++) {   /* bins: skipped (linear index queries) */
            uint32_t bin; int32_t n_chunk;
            ok = fread(&bin, 4, 1, f) == 1 && fread(&n_chunk, 4, 1, f) == 1 && n_chunk >= 0 &&
                 fseek(f, 16L * n_chunk, SEEK_CUR) == 0;
        }
        ok = ok && fread(&b->n_intv[r], 4, 1, f) == 1 && b->n_intv[r] >= 0;
        if (ok && b->n_intv[r]) {
            b->ioff[r] = (uint64_t *)malloc(8 * (size_t)b->n_intv[r]);
            ok = b->ioff[r] && fread(b->ioff[r], 8, (size_t)b->n_intv[r], f) == (size_t)b->n_intv[r];
        }
    }
    fclose(f);
    if (!ok) { bai_free(b); return NULL; }
    return b;
}

/* ---------------------------------------------------------------- one worker's reader */
typedef struct {
    int fd;
    bai_t *bai;
    z_stream zs;
    uint8_t cblk[65536 + 64];
    uint8_t ublk[65536];
    size_t ulen, upos;
    uint64_t next_coff;     /* file offset of the block after the current one */
    int eof;
    /* bam1_t-like record buffer */
    uint8_t *rec;
    size_t rec_cap;
    /* the window's reads (a single-contig pileup) */
    int32_t *pos, *endpos;
    uint64_t *cig_off;
    uint32_t *cigar;
    uint8_t *clip;
    int64_t n, cap;
    uint64_t ncig, cig_cap;
    int64_t tid_off[2];
    orc_pileup view;
    uint64_t stats[3];
    int err;
} reader_t;

static int load_block(reader_t *r, uint64_t coff) {
    uint8_t h[18];
    ssize_t got = pread(r->fd, h, 18, (off_t)coff);
    if (got == 0) { r->eof = 1; return 0; }
    if (got != 18 || h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) return -1;
    uint16_t xlen = rd16(h + 10);
    size_t bsize = 0;
    uint8_t x[256];
    if (xlen > sizeof x || pread(r->fd, x, xlen, (off_t)coff + 12) != xlen) return -1;
    for (size_t k = 0; k + 4 <= xlen;) {
        uint16_t slen = rd16(x + k + 2);
        if (x[k] == 66 && x[k + 1] == 67 && slen == 2) bsize = (size_t)rd16(x + k + 4) + 1;
        k += 4 + slen;
    }
    if (!bsize || bsize > sizeof r->cblk) return -1;
    if (pread(r->fd, r->cblk, bsize, (off_t)coff) != (ssize_t)bsize) return -1;
    const size_t cdata = 12 + xlen, clen = bsize - xlen - 20;
    const uint32_t isize = rd32(r->cblk + bsize - 4);
    if (isize > sizeof r->ublk) return -1;
    if (inflateReset(&r->zs) != Z_OK) return -1;
    r->zs.next_in = r->cblk + cdata;
    r->zs.avail_in = (uInt)clen;
    r->zs.next_out = r->ublk;
    r->zs.avail_out = (uInt)sizeof r->ublk;
    int rc = inflate(&r->zs, Z_FINISH);
    if (rc != Z_STREAM_END || r->zs.total_out != isize) return -1;
    r->ulen = isize;
    r->upos = 0;
    r->next_coff = coff + bsize;
    r->stats[0]++;
    r->stats[1] += isize;
    return 0;
}

/* read k bytes of the decompressed stream into dst; 1 = ok, 0 = clean EOF, -1 = error */
static int stream_read(reader_t *r, uint8_t *dst, size_t k) {
    while (k) {
        if (r->upos == r->ulen) {
            if (r->eof) return 0;
            if (load_block(r, r->next_coff)) return -1;
            if (r->eof || r->ulen == 0) { if (r->eof) return 0; continue; }
        }
        size_t t = r->ulen - r->upos;
        if (t > k) t = k;
        memcpy(dst, r->ublk + r->upos, t);
        r->upos += t; dst += t; k -= t;
    }
    return 1;
}

static int push_read(reader_t *r, int32_t pos, int32_t endp, const uint8_t *cig, uint32_t n, uint8_t clip) {
    if (r->n + 1 >= r->cap) {
        int64_t nc = r->cap ? 2 * r->cap : 256;
        int32_t *a = (int32_t *)realloc(r->pos, sizeof(int32_t) * (size_t)nc);
        if (!a) return -1;
        r->pos = a;
        if (!(a = (int32_t *)realloc(r->endpos, sizeof(int32_t) * (size_t)nc))) return -1;
        r->endpos = a;
        uint64_t *o = (uint64_t *)realloc(r->cig_off, sizeof(uint64_t) * (size_t)(nc + 1));
        if (!o) return -1;
        r->cig_off = o;
        uint8_t *c = (uint8_t *)realloc(r->clip, (size_t)nc);
        if (!c) return -1;
        r->clip = c;
        r->cap = nc;
    }
    if (r->ncig + n > r->cig_cap) {
        uint64_t nc = r->cig_cap ? r->cig_cap : 4096;
        while (nc < r->ncig + n) nc *= 2;
        uint32_t *c = (uint32_t *)realloc(r->cigar, sizeof(uint32_t) * (size_t)nc);
        if (!c) return -1;
        r->cigar = c;
        r->cig_cap = nc;
    }
    r->pos[r->n] = pos;
    r->endpos[r->n] = endp;
    r->clip[r->n] = clip;
    r->cig_off[r->n] = r->ncig;
    if (n) memcpy(r->cigar + r->ncig, cig, 4ull * n);
    r->ncig += n;
    r->n++;
    r->cig_off[r->n] = r->ncig;
    return 0;
}

/* htslib bam_tag2cigar's conditions: cigar[0] == <l_seq>S and a CG:B,I (or B,i) tag */
static int find_cg(const uint8_t *p, const uint8_t *end, const uint8_t **arr, uint32_t *cnt) {
    while (p + 3 <= end) {
        char t0 = (char)p[0], t1 = (char)p[1], ty = (char)p[2];
        p += 3;
        size_t sz = 0;
        switch (ty) {
        case 'A': case 'c': case 'C': sz = 1; break;
        case 's': case 'S': sz = 2; break;
        case 'i': case 'I': case 'f': sz = 4; break;
        case 'Z': case 'H':
            while (p < end && *p) p++;
            if (p >= end) return 0;
            p++;
            continue;
        case 'B': {
            if (p + 5 > end) return 0;
            char sub = (char)p[0];
            uint32_t n = rd32(p + 1);
            size_t es = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2
                        : (sub == 'i' || sub == 'I' || sub == 'f') ? 4 : 0;
            if (!es) return 0;
            if (t0 == 'C' && t1 == 'G') {
                if ((sub != 'I' && sub != 'i') || p + 5 + (size_t)n * 4 > end) return 0;
                *arr = p + 5;
                *cnt = n;
                return 1;
            }
            p += 5 + (size_t)n * es;
            continue;
        }
        default:
            return 0;
        }
        p += sz;
    }
    return 0;
}

/* sam_itr_queryi + sam_itr_next for (tid, [beg, end)): the yielded reads as a pileup */
static const orc_pileup *fetch_bgzf(void *ctx, int tid, int64_t beg, int64_t end, int64_t *lo, int64_t *hi) {
    reader_t *r = (reader_t *)ctx;
    r->n = 0;
    r->ncig = 0;
    *lo = *hi = 0;
    if (tid < 0 || tid >= r->bai->n_ref || end <= beg) return NULL;   /* hts_itr_query: no reads */
    const int64_t w = beg >> 14;
    if (w >= r->bai->n_intv[tid]) return NULL;   /* no read overlaps beg's window or any later one */
    const uint64_t voff = r->bai->ioff[tid][w];
    r->eof = 0;
    if (load_block(r, voff >> 16)) { r->err = 1; return NULL; }
    if (r->eof) return NULL;
    r->upos = (size_t)(voff & 0xffff);
    for (;;) {
        uint8_t bs4[4];
        int k = stream_read(r, bs4, 4);
        if (k <= 0) { if (k < 0) r->err = 1; break; }
        const uint32_t bs = rd32(bs4);
        if (bs < 32) { r->err = 1; break; }
        if (bs > r->rec_cap) {
            size_t nc = r->rec_cap ? r->rec_cap : 65536;
            while (nc < bs) nc *= 2;
            uint8_t *x = (uint8_t *)realloc(r->rec, nc);
            if (!x) { r->err = 1; break; }
            r->rec = x;
            r->rec_cap = nc;
        }
        if (stream_read(r, r->rec, bs) != 1) { r->err = 1; break; }   /* bam_read1: the whole record */
        r->stats[2]++;
        const uint8_t *b = r->rec, *bend = r->rec + bs;
        const int32_t rtid = (int32_t)rd32(b), rpos = (int32_t)rd32(b + 4);
        if (rtid != tid || (int64_t)rpos >= end) break;                 /* hts_itr_next: past the query */
        const uint32_t l_qname = b[8];
        const uint16_t n_cig = rd16(b + 12), flag = rd16(b + 14);
        const int32_t l_seq = (int32_t)rd32(b + 16);
        const uint8_t *qn = b + 32, *cg = qn + l_qname;
        if (l_seq < 0 || cg + 4ull * n_cig > bend) { r->err = 1; break; }
        const uint8_t *seq = cg + 4ull * n_cig, *aux = seq + (size_t)(l_seq + 1) / 2 + (size_t)l_seq;
        const uint8_t *cig = cg;
        uint32_t n = n_cig;
        if (n_cig > 0 && (rd32(cg) & 0xfu) == OP_S && (int64_t)(rd32(cg) >> 4) == l_seq && aux <= bend) {
            const uint8_t *arr;
            uint32_t cnt;
            if (find_cg(aux, bend, &arr, &cnt) && cnt >= n_cig && cnt < (1u << 29)) { cig = arr; n = cnt; }
        }
        int64_t rl = 0;   /* bam_endpos */
        if (!(flag & 4))
            for (uint32_t j = 0; j < n; j++) {
                const uint32_t w32 = rd32(cig + 4ull * j), op = w32 & 0xfu;
                if (op == OP_M || op == OP_D || op == OP_N || op == OP_EQ || op == OP_X) rl += w32 >> 4;
            }
        const int64_t endp = (int64_t)rpos + (rl ? rl : 1);
        if (endp <= beg) continue;
        /* the two soft-clip test words as the reference reads them through bam1_t.data */
        uint8_t clip = 0;
        if (n) {
            if ((rd32(cig + 4ull * (n - 1)) & 0xfu) == OP_S) clip |= 1;
            if ((rd32(cig) & 0xfu) == OP_S) clip |= 2;
        } else {
            const uint32_t padded = (l_qname + 3u) & ~3u;
            const uint8_t lastw0 = (padded >= 4 && padded - 4 < l_qname) ? qn[padded - 4] : 0;
            if ((lastw0 & 0xfu) == OP_S) clip |= 1;
            if (seq < bend && (seq[0] & 0xfu) == OP_S) clip |= 2;
        }
        if (push_read(r, rpos, (int32_t)endp, cig, n, clip)) { r->err = 1; break; }
    }
    r->tid_off[0] = 0;
    r->tid_off[1] = r->n;
    r->view.n_targets = 1;
    r->view.tid_off = r->tid_off;
    r->view.pos = r->pos;
    r->view.endpos = r->endpos;
    r->view.cig_off = r->cig_off;
    r->view.cigar = r->cigar;
    r->view.clip = r->clip;
    *lo = 0;
    *hi = r->n;
    return r->n ? &r->view : NULL;
}

typedef struct {
    const char *path;
    const orc_params *prm;
    const orc_locus *loci;
    orc_result *out;
    size_t n;
    int tix, nthreads;
    uint64_t stats[3];
    int err;
} job_t;

static void *worker(void *v) {
    job_t *j = (job_t *)v;
    reader_t *r = (reader_t *)calloc(1, sizeof(reader_t));
    if (!r) { j->err = 1; return NULL; }
    r->fd = open(j->path, O_RDONLY);        /* hts_open, per thread */
    r->bai = r->fd >= 0 ? bai_load(j->path) : NULL;   /* sam_index_load, per thread */
    if (r->fd < 0 || !r->bai || inflateInit2(&r->zs, -15) != Z_OK) {
        j->err = 1;
        if (r->fd >= 0) close(r->fd);
        bai_free(r->bai);
        free(r);
        return NULL;
    }
    /* A3's contig test is fetch_bgzf's; it hands the walk the yielded reads as a one-contig
     * pileup (the walk never looks at the contig again) */
    for (size_t i = (size_t)j->tix; i < j->n && !r->err; i += (size_t)j->nthreads)
        orc_refine_locus_src(fetch_bgzf, r, j->prm, &j->loci[i], &j->out[i], NULL);
    if (r->err) j->err = 1;
    memcpy(j->stats, r->stats, sizeof j->stats);
    inflateEnd(&r->zs);
    close(r->fd);
    bai_free(r->bai);
    free(r->rec); free(r->pos); free(r->endpos); free(r->cig_off); free(r->cigar); free(r->clip);
    free(r);
    return NULL;
}

int orc_bgzf_refine_batch(const char *bam_path, const orc_params *prm, const orc_locus *loci, size_t n,
                          orc_result *out, int threads, uint64_t *stats, char *err, size_t errcap) {
    if (threads < 1) threads = 1;
    job_t *jobs = (job_t *)calloc((size_t)threads, sizeof(job_t));
    pthread_t *th = (pthread_t *)calloc((size_t)threads, sizeof(pthread_t));
    if (!jobs || !th) { free(jobs); free(th); return -1; }
    for (int t = 0; t < threads; t++) {
        jobs[t] = (job_t){bam_path, prm, loci, out, n, t, threads, {0, 0, 0}, 0};
        if (threads == 1) worker(&jobs[t]);
        else pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    if (threads > 1)
        for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    int bad = 0;
    if (stats) memset(stats, 0, 3 * sizeof(uint64_t));
    for (int t = 0; t < threads; t++) {
        bad |= jobs[t].err;
        if (stats)
            for (int k = 0; k < 3; k++) stats[k] += jobs[t].stats[k];
    }
    free(jobs); free(th);
    if (bad && err && errcap) snprintf(err, errcap, "BGZF baseline: cannot read %s (+ .bai) or corrupt data", bam_path);
    return bad ? -1 : 0;
}
