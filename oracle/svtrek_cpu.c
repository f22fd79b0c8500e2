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
