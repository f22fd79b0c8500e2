/*
 * svtrek_cpu.c -- TEST INFRASTRUCTURE ONLY: the CPU restatement behind the product's C ABI.
 *
 * libsvtrek_cpu.so implements include/svtrek_gpu.h's host-buffer entry points on the oracle
 * (svtrek_oracle.c: the plain-C restatement of refinement.c / audit.c), so that parity
 * tests and the CPU baseline can link either backend through one ABI:
 * svt_open / svt_open_multi, svt_load_pileup (a deep copy), svt_refine_batch (pthread
 * workers, the tpool fan-out of audit.c:289-293), svt_count_work (the reference walk's
 * counters), svt_sliding_window_ins, svt_last_error, svt_close, svt_version, ...
 * Entry points that take device pointers or exist for the GPU's own machinery
 * (svt_refine_device*, svt_sync, the POA mode) return SVT_EINVAL here.  The product never
 * loads this library: svtrek_amd.Engine and the svtrek CLI bind libsvtrek_hip.so only.
 * Threads: SVTREK_CPU_THREADS, else the online CPU count.
 */
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <zlib.h>

#include "../include/svtrek_gpu.h"
#include "svtrek_oracle.h"

struct svt_ctx {
    svt_params prm;
    int threads;
    char err[256];
    int loaded;
    int32_t n_targets;
    int64_t *tid_off;
    int32_t *pos, *endpos;
    uint64_t *cig_off;
    uint32_t *cigar;
    uint8_t *clip;
    orc_pileup view;
    uint64_t bytes;
};

static svt_status fail(svt_ctx *c, svt_status s, const char *fmt, ...) {
    if (c) {
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(c->err, sizeof c->err, fmt, ap);
        va_end(ap);
    }
    return s;
}

static orc_params oparams(const svt_params *p) {
    orc_params o = {p->wider_interval, p->median_interval, p->narrow_interval, p->consensus_interval_range,
                    p->consensus_interval, p->consensus_min_count};
    return o;
}

static void drop(svt_ctx *c) {
    free(c->tid_off); free(c->pos); free(c->endpos); free(c->cig_off); free(c->cigar); free(c->clip);
    c->tid_off = NULL; c->pos = c->endpos = NULL; c->cig_off = NULL; c->cigar = NULL; c->clip = NULL;
    c->loaded = 0;
    c->bytes = 0;
}

svt_status svt_open(const svt_params *params, int device, svt_ctx **out) {
    (void)device;
    if (!params || !out) return SVT_EINVAL;
    if (params->consensus_min_count < 1) return SVT_EINVAL;   /* min_count <= 0 reads locations[-1] */
    svt_ctx *c = (svt_ctx *)calloc(1, sizeof(svt_ctx));
    if (!c) return SVT_ENOMEM;
    c->prm = *params;
    const char *t = getenv("SVTREK_CPU_THREADS");
    long n = t ? atol(t) : sysconf(_SC_NPROCESSORS_ONLN);
    c->threads = n < 1 ? 1 : (int)n;
    *out = c;
    return SVT_OK;
}

svt_status svt_open_multi(const svt_params *params, int device_count, const int *devices, svt_ctx **out) {
    if (device_count < 1) return SVT_EINVAL;
    return svt_open(params, devices ? devices[0] : 0, out);
}

int svt_device_count(const svt_ctx *ctx) { return ctx ? 1 : 0; }

svt_status svt_load_pileup(svt_ctx *c, const svt_pileup_view *v) {
    if (!c || !v || v->n_targets < 0 || (v->n_targets && (!v->tid_off || !v->cig_off)))
        return fail(c, SVT_EINVAL, "svt_load_pileup: bad view");
    drop(c);
    const int32_t nt = v->n_targets;
    const int64_t nr = nt ? v->tid_off[nt] : 0;
    const uint64_t nops = nr ? v->cig_off[nr] : 0;
    for (int32_t t = 0; t < nt; t++)
        if (v->tid_off[t + 1] < v->tid_off[t]) return fail(c, SVT_EINVAL, "svt_load_pileup: tid_off not monotone");
    c->tid_off = (int64_t *)malloc(sizeof(int64_t) * (size_t)(nt + 1));
    c->pos = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nr ? nr : 1));
    c->endpos = (int32_t *)malloc(sizeof(int32_t) * (size_t)(nr ? nr : 1));
    c->cig_off = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)(nr + 1));
    c->cigar = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(nops ? nops : 1));
    c->clip = v->clip ? (uint8_t *)malloc((size_t)(nr ? nr : 1)) : NULL;
    if (!c->tid_off || !c->pos || !c->endpos || !c->cig_off || !c->cigar || (v->clip && !c->clip)) {
        drop(c);
        return fail(c, SVT_ENOMEM, "svt_load_pileup: out of host memory");
    }
    if (nt) memcpy(c->tid_off, v->tid_off, sizeof(int64_t) * (size_t)(nt + 1));
    else c->tid_off[0] = 0;
    if (nr) {
        memcpy(c->pos, v->pos, sizeof(int32_t) * (size_t)nr);
        memcpy(c->endpos, v->endpos, sizeof(int32_t) * (size_t)nr);
        memcpy(c->cig_off, v->cig_off, sizeof(uint64_t) * (size_t)(nr + 1));
        if (v->clip) memcpy(c->clip, v->clip, (size_t)nr);
    } else {
        c->cig_off[0] = 0;
    }
    if (nops) memcpy(c->cigar, v->cigar, sizeof(uint32_t) * (size_t)nops);
    c->n_targets = nt;
    c->view = (orc_pileup){nt, c->tid_off, c->pos, c->endpos, c->cig_off, c->cigar, c->clip};
    c->bytes = (uint64_t)nr * 17 + nops * 4 + (uint64_t)(nt + 1) * 8;
    c->loaded = 1;
    return SVT_OK;
}

svt_status svt_refine_batch(svt_ctx *c, const svt_locus *loci, size_t n, svt_result *out) {
    if (!c) return SVT_EINVAL;
    if (!c->loaded) return fail(c, SVT_ESTATE, "svt_refine_batch before svt_load_pileup");
    if (n == 0) return SVT_OK;
    if (!loci || !out) return fail(c, SVT_EINVAL, "svt_refine_batch: NULL buffers");
    const orc_params p = oparams(&c->prm);
    if (orc_refine_batch(&c->view, &p, (const orc_locus *)loci, n, (orc_result *)out, c->threads, NULL))
        return fail(c, SVT_ENOMEM, "svt_refine_batch: out of host memory");
    return SVT_OK;
}

svt_status svt_count_work(svt_ctx *c, const svt_locus *loci, size_t n, svt_work *out) {
    if (!c || !out) return SVT_EINVAL;
    if (!c->loaded) return fail(c, SVT_ESTATE, "svt_count_work before svt_load_pileup");
    memset(out, 0, sizeof *out);
    if (n == 0) return SVT_OK;
    const orc_params p = oparams(&c->prm);
    orc_result *tmp = (orc_result *)malloc(sizeof(orc_result) * n);
    orc_work w;
    if (!tmp || orc_refine_batch(&c->view, &p, (const orc_locus *)loci, n, tmp, c->threads, &w)) {
        free(tmp);
        return fail(c, SVT_ENOMEM, "svt_count_work: out of host memory");
    }
    free(tmp);
    out->windows = w.windows;
    out->reads = w.reads;
    out->ops_walked = w.ops_walked;
    out->candidates = w.candidates;
    out->event_bytes = 24ull * n + 12ull * w.reads + 4ull * w.ops_walked;   /* the reference walk's bytes */
    return SVT_OK;
}

uint64_t svt_sw_subwindows(const svt_sw_query *q, int32_t window_size) {
    if (!q || window_size < 1 || q->end <= q->start) return 0;
    return ((uint64_t)q->end - q->start + (uint64_t)window_size - 1) / (uint64_t)window_size;
}

svt_status svt_sliding_window_ins(svt_ctx *c, const svt_sw_query *q, size_t n, int32_t window_size,
                                  int32_t slide_size, int32_t *best, svt_sw_window *sub) {
    if (!c) return SVT_EINVAL;
    if (!c->loaded) return fail(c, SVT_ESTATE, "svt_sliding_window_ins before svt_load_pileup");
    if (window_size < 1 || slide_size < 1) return fail(c, SVT_EINVAL, "window_size and slide_size must be >= 1");
    if (n && (!q || !best)) return fail(c, SVT_EINVAL, "NULL buffers");
    uint64_t k = 0;
    for (size_t i = 0; i < n; i++) {
        if ((uint64_t)q[i].end + (uint64_t)window_size > (1ull << 32))
            return fail(c, SVT_EINVAL, "end + window_size > 2^32 (the reference's sub_start wraps)");
        const uint64_t m = svt_sw_subwindows(&q[i], window_size);
        int32_t *cand = (int32_t *)malloc(sizeof(int32_t) * (size_t)(m ? m : 1));
        int32_t *sup = (int32_t *)malloc(sizeof(int32_t) * (size_t)(m ? m : 1));
        if (!cand || !sup) { free(cand); free(sup); return fail(c, SVT_ENOMEM, "out of host memory"); }
        best[i] = orc_sliding_window_ins(&c->view, q[i].chrom, q[i].start, q[i].end, window_size, slide_size,
                                         c->prm.consensus_min_count, cand, sup);
        if (sub)
            for (uint64_t j = 0; j < m; j++) sub[k + j] = (svt_sw_window){cand[j], sup[j]};
        k += m;
        free(cand); free(sup);
    }
    return SVT_OK;
}

/* device-pointer and GPU-machinery entry points: not in the CPU backend */
svt_status svt_refine_device(svt_ctx *c, const svt_locus *d_loci, size_t n, svt_result *d_out, void *s) {
    (void)d_loci; (void)n; (void)d_out; (void)s;
    return fail(c, SVT_EINVAL, "svt_refine_device: no device memory in the CPU backend");
}
svt_status svt_refine_device_records(svt_ctx *c, const svt_locus *d_loci, size_t n, const uint32_t *d_index,
                                     uint32_t base, svt_record *d_out, void *s) {
    (void)d_loci; (void)n; (void)d_out; (void)base; (void)d_index; (void)s;
    return fail(c, SVT_EINVAL, "svt_refine_device_records: no device memory in the CPU backend");
}
svt_status svt_sync(svt_ctx *c, void *s) { (void)s; return c ? SVT_OK : SVT_EINVAL; }
/* the CPU backend walks every read per query: it has no device index to rebuild */
svt_status svt_reindex(svt_ctx *c, void *s) {
    (void)s;
    if (!c) return SVT_EINVAL;
    return c->loaded ? SVT_OK : fail(c, SVT_ESTATE, "svt_reindex before svt_load_pileup");
}
void svt_poa_default_params(svt_poa_params *p) { if (p) memset(p, 0, sizeof *p); }
uint64_t svt_pileup_ins_count(const svt_ctx *c) { (void)c; return 0; }
svt_status svt_load_insseq(svt_ctx *c, const svt_insseq_view *s) {
    (void)s;
    return fail(c, SVT_EINVAL, "svt_load_insseq: the POA mode is GPU-only (oracle/poa_oracle.c is its checker)");
}
svt_status svt_poa_consensus(svt_ctx *c, const svt_poa_params *p, const svt_locus *loci, const svt_result *res,
                             size_t n, int32_t cap, uint8_t *bases, svt_poa_result *out) {
    (void)p; (void)loci; (void)res; (void)n; (void)out; (void)bases; (void)cap;
    return fail(c, SVT_EINVAL, "svt_poa_consensus: the POA mode is GPU-only");
}
uint64_t svt_poa_deferred(const svt_ctx *c) { (void)c; return 0; }
uint64_t svt_pileup_device_bytes(const svt_ctx *c) { return c ? c->bytes : 0; }
svt_status svt_last_load_stats(const svt_ctx *c, svt_load_stats *out) {
    if (!c || !out) return SVT_EINVAL;
    memset(out, 0, sizeof *out);
    return SVT_OK;
}
/* BGZF inflate with zlib (raw DEFLATE), block by block: the CPU side of svt_bgzf_inflate. */
static uint32_t cpu_inflate(const uint8_t *comp, const svt_bgzf_block *b, size_t n, uint8_t *out) {
    z_stream zs;
    memset(&zs, 0, sizeof zs);
    if (inflateInit2(&zs, -15) != Z_OK) return 0;
    uint32_t bad = 0xffffffffu;
    for (size_t i = 0; i < n && bad == 0xffffffffu; i++) {
        inflateReset(&zs);
        zs.next_in = (Bytef *)(comp + b[i].coff);
        zs.avail_in = b[i].clen;
        zs.next_out = out + b[i].uoff;
        zs.avail_out = b[i].ulen;
        if (inflate(&zs, Z_FINISH) != Z_STREAM_END || zs.total_out != b[i].ulen) bad = (uint32_t)i;
    }
    inflateEnd(&zs);
    return bad;
}
static uint32_t cpu_inflate_bad = 0xffffffffu;
svt_status svt_bgzf_inflate(svt_ctx *c, const uint8_t *comp, size_t comp_bytes, const svt_bgzf_block *b, size_t n,
                            uint8_t *out, size_t out_bytes) {
    if (!c) return SVT_EINVAL;
    for (size_t i = 0; i < n; i++)
        if (b[i].clen > 65536u || b[i].ulen > 65536u || b[i].coff > comp_bytes || b[i].clen > comp_bytes - b[i].coff ||
            b[i].uoff > out_bytes || b[i].ulen > out_bytes - b[i].uoff)
            return fail(c, SVT_EINVAL, "BGZF block outside its buffers (or over 64 KiB)");
    const uint32_t bad = cpu_inflate(comp, b, n, out);
    return bad == 0xffffffffu ? SVT_OK : fail(c, SVT_EINVAL, "corrupt BGZF block %u (does not inflate to its ISIZE)", bad);
}
svt_status svt_bgzf_inflate_device(svt_ctx *c, const uint8_t *d_comp, const svt_bgzf_block *d_blocks, size_t n,
                                   uint8_t *d_out, void *s) {   /* host memory stands in for device memory here */
    (void)s;
    if (!c) return SVT_EINVAL;
    cpu_inflate_bad = cpu_inflate(d_comp, d_blocks, n, d_out);
    return SVT_OK;
}
svt_status svt_bgzf_inflate_status(svt_ctx *c, void *s, uint32_t *bad) {
    (void)s;
    if (!c || !bad) return SVT_EINVAL;
    *bad = cpu_inflate_bad;
    return *bad == 0xffffffffu ? SVT_OK : fail(c, SVT_EINVAL, "corrupt BGZF block %u", *bad);
}
double svt_bgzf_last_inflate_ms(const svt_ctx *c) { (void)c; return 0.0; }
void *svt_host_alloc(svt_ctx *c, size_t bytes) { (void)c; return malloc(bytes ? bytes : 1); }
void svt_host_free(svt_ctx *c, void *p) { (void)c; free(p); }

const char *svt_last_error(const svt_ctx *c) { return c ? c->err : "NULL context"; }
void svt_close(svt_ctx *c) {
    if (!c) return;
    drop(c);
    free(c);
}
const char *svt_version(void) { return "svtrek_cpu (oracle restatement, test infrastructure)"; }

/* ---- svt_bam_dec_*: the BAM decoded record by record on the host (a plain-C restatement of
 * htslib's bam_read1 + bam_tag2cigar for the fields the path reads, refinement.c:117-120), so
 * that the CLI's decode flow runs on this backend too and cross-checks the device decoder. */
struct svt_bam_dec {
    svt_ctx *c;
    int32_t n_ref;
    int first;
    uint8_t *buf;              /* inflated bytes not consumed yet (an incomplete record) */
    size_t n, cap;
    int32_t *tid, *pos, *endpos;
    uint8_t *clip;
    uint64_t *cig_off;
    uint32_t *cigar;
    size_t nr, rcap, nw, wcap;
    svt_bam_dec_stats st;
};

static uint32_t bd_rd32(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
static uint32_t bd_rd16(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8; }

/* the CG:B,I array of a record's aux fields (htslib bam_tag2cigar's lookup) */
static int bd_find_cg(const uint8_t *p, const uint8_t *end, const uint8_t **arr, uint32_t *cnt) {
    while (p + 3 <= end) {
        const char t0 = (char)p[0], t1 = (char)p[1], ty = (char)p[2];
        p += 3;
        if (ty == 'A' || ty == 'c' || ty == 'C') { p += 1; continue; }
        if (ty == 's' || ty == 'S') { p += 2; continue; }
        if (ty == 'i' || ty == 'I' || ty == 'f') { p += 4; continue; }
        if (ty == 'Z' || ty == 'H') {
            while (p < end && *p) p++;
            if (p >= end) return 0;
            p++;
            continue;
        }
        if (ty != 'B' || p + 5 > end) return 0;
        const char sub = (char)p[0];
        const uint32_t n = bd_rd32(p + 1);
        const size_t es = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2
                          : (sub == 'i' || sub == 'I' || sub == 'f') ? 4 : 0;
        if (!es) return 0;
        if (t0 == 'C' && t1 == 'G') {
            if ((sub != 'I' && sub != 'i') || p + 5 + (size_t)n * 4 > end) return 0;
            *arr = p + 5;
            *cnt = n;
            return 1;
        }
        p += 5 + (size_t)n * es;
    }
    return 0;
}

static int bd_grow(void **p, size_t *cap, size_t need, size_t elem) {
    if (need <= *cap) return 1;
    size_t nc = *cap ? *cap : 1024;
    while (nc < need) nc += nc / 2 + 1;
    void *q = realloc(*p, nc * elem);
    if (!q) return 0;
    *p = q;
    *cap = nc;
    return 1;
}

/* One complete record (r: after its block_size word) -> the columns; 0 = corrupt. */
static int bd_take(svt_bam_dec *d, const uint8_t *r, uint32_t bs) {
    const uint8_t *rend = r + bs;
    const int32_t tid = (int32_t)bd_rd32(r), pos = (int32_t)bd_rd32(r + 4);
    const uint32_t l_qname = r[8], n_cig = bd_rd16(r + 12), flag = bd_rd16(r + 14);
    const int32_t l_seq = (int32_t)bd_rd32(r + 16);
    d->st.records++;
    if (!(tid >= 0 && tid < d->n_ref && pos >= 0)) return 1;   /* no tid >= 0 query yields it */
    const uint8_t *qn = r + 32, *cg = qn + l_qname;
    if (cg + 4ull * n_cig > rend || l_seq < 0) return 0;
    const uint8_t *after = cg + 4ull * n_cig, *aux = after + (size_t)(l_seq + 1) / 2 + (size_t)l_seq;
    const uint8_t *cig = cg;
    uint32_t n = n_cig;
    if (n_cig > 0 && (bd_rd32(cg) & 0xfu) == 4u && (int64_t)(bd_rd32(cg) >> 4) == l_seq && aux <= rend) {
        const uint8_t *arr;
        uint32_t cnt;
        if (bd_find_cg(aux, rend, &arr, &cnt) && cnt >= n_cig && cnt < (1u << 29)) { cig = arr; n = cnt; d->st.cg_restored++; }
    }
    uint8_t clip = 0;   /* the words refinement.c:120 and :210 test (the padded name / first SEQ byte for n == 0) */
    if (n) {
        if ((bd_rd32(cig + 4ull * (n - 1)) & 0xfu) == 4u) clip |= SVT_CLIP_LAST_S;
        if ((bd_rd32(cig) & 0xfu) == 4u) clip |= SVT_CLIP_FIRST_S;
    } else {
        const uint32_t padded = (l_qname + 3u) & ~3u;
        const uint8_t w0 = (padded >= 4 && padded - 4 < l_qname) ? qn[padded - 4] : 0;
        if ((w0 & 0xfu) == 4u) clip |= SVT_CLIP_LAST_S;
        if (after < rend && (after[0] & 0xfu) == 4u) clip |= SVT_CLIP_FIRST_S;
    }
    if (d->nr + 1 > d->rcap) {   /* every per-read column to the same capacity */
        const size_t nc = d->rcap ? d->rcap + d->rcap / 2 : 1024;
        int32_t *t = (int32_t *)realloc(d->tid, nc * sizeof(int32_t));
        if (t) d->tid = t;
        int32_t *ps = (int32_t *)realloc(d->pos, nc * sizeof(int32_t));
        if (ps) d->pos = ps;
        int32_t *ep = (int32_t *)realloc(d->endpos, nc * sizeof(int32_t));
        if (ep) d->endpos = ep;
        uint8_t *cl = (uint8_t *)realloc(d->clip, nc);
        if (cl) d->clip = cl;
        uint64_t *co = (uint64_t *)realloc(d->cig_off, nc * sizeof(uint64_t));
        if (co) d->cig_off = co;
        if (!t || !ps || !ep || !cl || !co) return 0;
        d->rcap = nc;
    }
    if (!bd_grow((void **)&d->cigar, &d->wcap, d->nw + n + 1, 4)) return 0;
    int64_t rl = 0;
    for (uint32_t j = 0; j < n; j++) {
        const uint32_t w = bd_rd32(cig + 4ull * j), op = w & 0xfu;
        d->cigar[d->nw + j] = w;
        if (!(flag & 4) && (op == 0 || op == 2 || op == 3 || op == 7 || op == 8)) rl += w >> 4;
    }
    d->tid[d->nr] = tid;
    d->pos[d->nr] = pos;
    d->endpos[d->nr] = (int32_t)(pos + (rl ? rl : 1));   /* htslib bam_endpos */
    d->clip[d->nr] = clip;
    d->cig_off[d->nr] = d->nw;
    d->nr++;
    d->nw += n;
    d->st.reads++;
    d->st.cigar_ops += n;
    return 1;
}

svt_status svt_bam_dec_open(svt_ctx *c, int32_t n_targets, svt_bam_dec **out) {
    if (!c || !out || n_targets < 0) return SVT_EINVAL;
    svt_bam_dec *d = (svt_bam_dec *)calloc(1, sizeof *d);
    if (!d) return fail(c, SVT_ENOMEM, "out of host memory");
    d->c = c;
    d->n_ref = n_targets;
    d->first = 1;
    *out = d;
    return SVT_OK;
}

svt_status svt_bam_dec_feed(svt_bam_dec *d, const uint8_t *comp, size_t comp_bytes, const svt_bgzf_block *b, size_t n,
                            uint64_t skip) {
    if (!d) return SVT_EINVAL;
    svt_ctx *c = d->c;
    uint64_t U = 0;
    for (size_t i = 0; i < n; i++) {
        if (b[i].clen > 65536u || b[i].ulen > 65536u || b[i].coff > comp_bytes || b[i].clen > comp_bytes - b[i].coff)
            return fail(c, SVT_EINVAL, "BGZF block outside its buffers (or over 64 KiB)");
        if (b[i].uoff + b[i].ulen > U) U = b[i].uoff + b[i].ulen;
    }
    if (!bd_grow((void **)&d->buf, &d->cap, d->n + U + 1, 1)) return fail(c, SVT_ENOMEM, "out of host memory");
    const uint32_t bad = cpu_inflate(comp, b, n, d->buf + d->n);
    if (bad != 0xffffffffu) return fail(c, SVT_EINVAL, "corrupt BGZF block %u of the batch (does not inflate to its ISIZE)", bad);
    size_t N = d->n + U, p = d->first ? (size_t)skip : 0;
    if (p > N) return fail(c, SVT_EINVAL, "BAM decode: the header runs past the first batch");
    while (p + 4 <= N) {   /* the record chain: block_size hops */
        const uint32_t bs = bd_rd32(d->buf + p);
        if (bs < 32) return fail(c, SVT_EINVAL, "corrupt BAM record (block_size < 32)");
        if (p + 4 + bs > N) break;
        if (!bd_take(d, d->buf + p + 4, bs)) return fail(c, SVT_EINVAL, "corrupt BAM record");
        p += 4 + (size_t)bs;
    }
    memmove(d->buf, d->buf + p, N - p);
    d->n = N - p;
    d->first = 0;
    d->st.batches++;
    d->st.inflated_bytes += U;
    return SVT_OK;
}

svt_status svt_bam_dec_stats_get(const svt_bam_dec *d, svt_bam_dec_stats *out) {
    if (!d || !out) return SVT_EINVAL;
    *out = d->st;
    return SVT_OK;
}

static const svt_bam_dec *bd_sort_ctx;
static int bd_cmp(const void *a, const void *b) {   /* by (tid, pos), then input order (stable) */
    const size_t x = *(const size_t *)a, y = *(const size_t *)b;
    const svt_bam_dec *d = bd_sort_ctx;
    if (d->tid[x] != d->tid[y]) return d->tid[x] < d->tid[y] ? -1 : 1;
    if (d->pos[x] != d->pos[y]) return d->pos[x] < d->pos[y] ? -1 : 1;
    return x < y ? -1 : x > y;
}

svt_status svt_bam_dec_load(svt_bam_dec *d) {
    if (!d) return SVT_EINVAL;
    svt_ctx *c = d->c;
    if (d->n) return fail(c, SVT_EINVAL, "truncated BAM record at end of file");
    const size_t nr = d->nr;
    size_t *idx = (size_t *)malloc(sizeof(size_t) * (nr ? nr : 1));
    int64_t *toff = (int64_t *)calloc((size_t)d->n_ref + 1, sizeof(int64_t));
    int32_t *pos = (int32_t *)malloc(sizeof(int32_t) * (nr ? nr : 1)), *end = (int32_t *)malloc(sizeof(int32_t) * (nr ? nr : 1));
    uint8_t *clip = (uint8_t *)malloc(nr ? nr : 1);
    uint64_t *off = (uint64_t *)malloc(sizeof(uint64_t) * (nr + 1));
    uint32_t *cig = (uint32_t *)malloc(4 * (d->nw ? d->nw : 1));
    svt_status s = SVT_ENOMEM;
    if (idx && toff && pos && end && clip && off && cig) {
        for (size_t i = 0; i < nr; i++) idx[i] = i;
        bd_sort_ctx = d;
        qsort(idx, nr, sizeof(size_t), bd_cmp);   /* the host ingest's order: sorted by (tid, pos), stable */
        uint64_t w = 0;
        for (size_t k = 0; k < nr; k++) {
            const size_t i = idx[k];
            const uint64_t o = d->cig_off[i], m = (i + 1 < nr ? d->cig_off[i + 1] : d->nw) - o;
            pos[k] = d->pos[i]; end[k] = d->endpos[i]; clip[k] = d->clip[i];
            off[k] = w;
            if (m) memcpy(cig + w, d->cigar + o, 4 * m);
            w += m;
            toff[d->tid[i] + 1]++;
        }
        off[nr] = w;
        for (int32_t t = 0; t < d->n_ref; t++) toff[t + 1] += toff[t];
        svt_pileup_view v = {d->n_ref, toff, pos, end, off, cig, clip};
        s = svt_load_pileup(c, &v);
    } else {
        fail(c, SVT_ENOMEM, "out of host memory");
    }
    free(idx); free(toff); free(pos); free(end); free(clip); free(off); free(cig);
    return s;
}

void svt_bam_dec_close(svt_bam_dec *d) {
    if (!d) return;
    free(d->buf); free(d->tid); free(d->pos); free(d->endpos); free(d->clip); free(d->cig_off); free(d->cigar);
    free(d);
}
