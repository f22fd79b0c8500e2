/*
 * svtrek_oracle.h -- TEST INFRASTRUCTURE ONLY (the parity checker), never shipped.
 *
 * A clean-room CPU restatement of SVTrek's `audt` hot path (reference
 * audit.c / refinement.c / utils.c), used by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg -- nothing else may load it.  See svtrek_oracle.c for
 * the per-function reference citations and DESIGN.md "Oracle" for how it is pinned.
 */
#ifndef SVTREK_ORACLE_H
#define SVTREK_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same field meaning as svt_params / svt_locus / svt_result / svt_pileup_view
 * (include/svtrek_gpu.h); restated here so the oracle does not depend on the product. */
typedef struct orc_params {
    int32_t wider_interval, median_interval, narrow_interval;
    int32_t consensus_interval_range, consensus_interval, consensus_min_count;
} orc_params;

typedef struct orc_locus  { int32_t type, chrom; uint32_t pos, end; } orc_locus;
typedef struct orc_result { uint32_t start, end; } orc_result;

typedef struct orc_pileup {
    int32_t         n_targets;
    const int64_t  *tid_off;
    const int32_t  *pos;
    const int32_t  *endpos;
    const uint64_t *cig_off;
    const uint32_t *cigar;
    const uint8_t  *clip;     /* bit0: op(cigar[n-1])==S, bit1: op(cigar[0])==S; NULL = derive */
} orc_pileup;

typedef struct orc_work { uint64_t windows, reads, ops_walked, candidates; } orc_work;

int  orc_lower_bound(const int *arr, int size, int location);
int  orc_upper_bound(const int *arr, int size, int location);
void orc_sort_ints(int *arr, int n);
int  orc_consensus_pos(int *locations, int size, int pos, int min_count, int ci, int range);

/* window scans; sv_type as reference sv_type_t (1 INS, 2 DEL, 3 INV) */
int orc_refine_start(const orc_pileup *p, int sv_type, int chrom, uint32_t s, uint32_t e,
                     uint32_t imprecise_pos, const orc_params *prm, orc_work *w);
int orc_refine_end  (const orc_pileup *p, int sv_type, int chrom, uint32_t s, uint32_t e,
                     uint32_t imprecise_pos, const orc_params *prm, orc_work *w);
int orc_refine_point(const orc_pileup *p, int sv_type, int chrom, uint32_t s, uint32_t e,
                     uint32_t imprecise_pos, const orc_params *prm, orc_work *w);
int orc_refine_ins  (const orc_pileup *p, int chrom, uint32_t s, uint32_t e,
                     uint32_t imprecise_pos, const orc_params *prm, orc_work *w);

/* A read source for one region query (A3): returns a pileup and the range [*lo, *hi) of
 * its reads that holds every read yielded for (tid, [beg, end)) -- a superset is fine, the
 * walk applies the yield test (pos < end && endpos > beg) itself; NULL = no reads. */
typedef const orc_pileup *(*orc_fetch_fn)(void *ctx, int tid, int64_t beg, int64_t end, int64_t *lo, int64_t *hi);
/* A2 + A4..A10 of one record with reads from `fetch` (the in-memory pileup, or
 * bgzf_ref.c's per-query BGZF reader). */
void orc_refine_locus_src(orc_fetch_fn fetch, void *ctx, const orc_params *prm, const orc_locus *l,
                          orc_result *r, orc_work *w);

/* The reference-shaped CPU baseline (bgzf_ref.c): `threads` workers, each
 * with its own file handle and its own copy of the BAI (audit.c:269-272), every region query
 * seeking to the BAI's linear-index offset and inflating + decoding the BGZF blocks from
 * there (htslib's sam_itr_queryi/sam_itr_next with no block cache, refinement.c:114-117).
 * Loci are handed out in VCF order.  0 on success; -1 on an I/O / format error (message in
 * err).  stats (may be NULL): [0] blocks inflated, [1] bytes inflated, [2] records decoded. */
int orc_bgzf_refine_batch(const char *bam_path, const orc_params *prm, const orc_locus *loci, size_t n,
                          orc_result *out, int threads, uint64_t *stats, char *err, size_t errcap);

/* A2 windows + A4..A7 for one parsed record (the deletion/insertion/inversion wrappers). */
void orc_refine_locus(const orc_pileup *p, const orc_params *prm, const orc_locus *l,
                      orc_result *r, orc_work *w);
/* Batch over n loci with `threads` pthread workers (the tpool fan-out of audit.c:289-293). */
int  orc_refine_batch(const orc_pileup *p, const orc_params *prm, const orc_locus *loci,
                      size_t n, orc_result *out, int threads, orc_work *w);

/* sliding_window_ins (sliding_window.c:8-97; dead code in the reference -- no caller).
 * Sub-windows [s, min(s+ws, end)) for s = start, start+ws, ... < end; per sub-window the
 * INS walk of refine_ins and a sliding-support vote.  sub_cand/sub_support (may be NULL)
 * receive each sub-window's bestCandidate (-1: none / no line printed) and maxSupport;
 * returns bestCandidateOverall.  Requires ws >= 1, slide >= 1, end + ws <= 2^32. */
int orc_sliding_window_ins(const orc_pileup *p, int chrom, uint32_t start, uint32_t end, int window_size,
                           int slide_size, int min_count, int32_t *sub_cand, int32_t *sub_support);

/* Allele consensus (POA; no reference behaviour -- parity unpinned, see poa_oracle.c). */
typedef struct orc_poa_params {
    int32_t match, mismatch, gap_open, gap_ext;   /* 2, 4, 4, 2 */
    int32_t band_b, band_f_permille;              /* band w = b + f*len: 10, 10 (= 0.01) */
    int32_t max_seqs, max_len, max_nodes;         /* 32, 4000, 32768 */
    int32_t support_radius, max_support;          /* 20, 64 */
} orc_poa_params;

/* Consensus of nseq nt4 sequences (bases[off[i] .. off[i+1])), in order; returns its
 * length (written up to cap), -1 on allocation failure; *nused = sequences fused. */
int orc_poa_consensus(const uint8_t *bases, const uint64_t *off, int nseq, const orc_poa_params *pp,
                      uint8_t *out, int cap, int32_t *nused);
/* Supporting I ops (global indices into the insertion-sequence arrays) of an INS call
 * refined to `refined` over window [s, e]; returns the count (first cap written). */
int orc_poa_support(const orc_pileup *p, const uint64_t *ins_base, int chrom, uint32_t s, uint32_t e,
                    uint32_t refined, const orc_poa_params *pp, int64_t *idx, int cap);

/* A1: parse one VCF data line (modified in place, as strtok_r does).  Returns
 * 1 = record reaches the type switch (*l filled), 0 = skipped silently,
 * 2 = skipped with a stderr message (text copied into err). */
int orc_parse_line(char *line, orc_locus *l, char *err, size_t errcap);

/* A11: the stdout text the reference prints for one record (0 bytes for
 * DUP/TRA/BND/unknown, whose "[ERROR] Unkown type." goes to stderr). */
int orc_format_result(const orc_locus *l, const orc_result *r, char *buf, size_t cap);

/* End to end: VCF text -> the reference's stdout text, records in VCF order,
 * framed by the two [INFO] lines.  *out is malloc'ed; free with orc_free. */
int  orc_audit_text(const char *vcf, size_t vcf_len, const orc_pileup *p,
                    const orc_params *prm, char **out, size_t *out_len);
void orc_free(void *ptr);

#ifdef __cplusplus
}
#endif
#endif
