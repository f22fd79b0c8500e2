/*
 * svtrek_gpu.h -- C ABI of the MI355X SV-refinement engine (the `audt` hot path).
 *
 * This header is the drop-in boundary.  The reference has no FFI: its hot path is
 * three internal C calls made once per VCF record by the worker `thread_func`
 * (reference audit.c:50-248):
 *
 *   void deletion (int chrom, interval begin, interval end, interval sv_inter,
 *                  t_arg *params, interval *res_inter);          refinement.h:59 / refinement.c:327-330
 *   void insertion(int chrom, interval begin, uint32_t pos,
 *                  t_arg *params, uint32_t *res_start);           refinement.h:76 / refinement.c:332-334
 *   void inversion(int chrom, interval begin, interval end, interval sv_inter,
 *                  t_arg *params, interval *res_inter);           refinement.h:94 / refinement.c:336-339
 *
 * each of which runs htslib region queries (sam_itr_queryi/sam_itr_next,
 * refinement.c:114-117), a CIGAR walk (refinement.c:103-325) and the consensus vote
 * (consensus_pos, refinement.c:41-101).  Here the per-record calls become ONE
 * batched call over many loci (svt_refine_batch / svt_refine_device); the reads the
 * htslib iterator would yield come from a columnar pileup loaded once
 * (svt_load_pileup), and the window arithmetic of audit.c:176-232 happens inside
 * the engine from the parsed record (svt_locus) and the parameters (svt_params =
 * the six refinement fields of t_arg, params.h:81-87).
 *
 * Conventions: plain C types only, no HIP/torch types; every function returns 0
 * (SVT_OK) or a negative svt_status; no exceptions cross the ABI.  A context is used by
 * one host thread at a time (like the reference's per-worker t_arg, audit.c:269-285);
 * every entry point selects the context's device itself and restores the calling
 * thread's current device before returning, so one thread may drive several contexts on
 * several GPUs.  A context opened with svt_open_multi spreads svt_refine_batch /
 * svt_count_work / svt_sliding_window_ins over its devices internally (the pileup is
 * replicated: it is a few GB against 288 GB of HBM per MI355X).  Launches of one context
 * execute in submission order even when issued on different streams (the context
 * inserts the stream dependency; the spill pool and the work counters are per context).
 * Results use the reference's encoding: a breakpoint the vote could not refine is
 * 0xFFFFFFFF (refinement.c returns -1, stored into uint32 at audit.c:179,194).
 */
#ifndef SVTREK_GPU_H
#define SVTREK_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t svt_status;
#define SVT_OK        0
#define SVT_EINVAL   -1   /* bad argument (NULL, min_count < 1, malformed pileup)   */
#define SVT_EDEVICE  -2   /* HIP runtime error (no device, launch failure)           */
#define SVT_ENOMEM   -3   /* device or host allocation failed                        */
#define SVT_ESTATE   -4   /* call out of order (refine before load_pileup)           */
#define SVT_EOVERFLOW -5  /* candidate spill pool exhausted; raise spill_bytes       */

/* SV type codes: identical values to the reference's sv_type_t (params.h:113-121). */
#define SVT_UNKNOWN 0
#define SVT_INS     1
#define SVT_DEL     2
#define SVT_INV     3
#define SVT_DUP     4
#define SVT_TRA     5
#define SVT_BND     6

#define SVT_NA 0xFFFFFFFFu        /* "not refined" (printed as NA, audit.c:181,197)   */

/* Refinement knobs -- the t_arg fields of params.h:81-87; defaults params.h:27-32. */
typedef struct svt_params {
    int32_t wider_interval;            /* --wider-interval            (20000) */
    int32_t median_interval;           /* --median-interval           (10000) */
    int32_t narrow_interval;           /* --narrow-interval           ( 2000) */
    int32_t consensus_interval_range;  /* --consensus-interval-range  (  500) */
    int32_t consensus_interval;        /* --consensus-interval        (    5) */
    int32_t consensus_min_count;       /* --consensus-min-count       (    3), must be >= 1 */
    uint64_t spill_bytes;              /* device pool for windows with > SVT_LDS_CANDS
                                          candidates; 0 = default (64 MiB)            */
} svt_params;

/* One parsed VCF record as it reaches the type switch of audit.c:175.
 * chrom = chrom_index of audit.c:101-105 (the BAM tid is chrom-1, refinement.c:114);
 * pos/end are the uint32 values of audit.c:108 and audit.c:159/165. */
typedef struct svt_locus {
    int32_t  type;   /* SVT_INS / SVT_DEL / SVT_INV (others yield NA/NA)           */
    int32_t  chrom;
    uint32_t pos;
    uint32_t end;
} svt_locus;

/* Refined breakpoints.  DEL: {refine_start, refine_end}; INS: {refine_ins, NA};
 * INV: {refine_point, refine_point} (always NA, refinement.c:250). */
typedef struct svt_result {
    uint32_t start;
    uint32_t end;
} svt_result;

/* Soft-clip tests the reference makes on every yielded read, precomputed at ingest so
 * reads with n_cigar == 0 keep the bytes the reference actually tests
 * (refinement.c:120 reads cigar[n_cigar-1], refinement.c:210 reads cigar[0]). */
#define SVT_CLIP_LAST_S  0x1u   /* bam_cigar_op(cigar[n_cigar-1]) == S  */
#define SVT_CLIP_FIRST_S 0x2u   /* bam_cigar_op(cigar[0])         == S  */

/* Caller-owned columnar pileup: the records htslib's iterator can yield, i.e. every
 * BAM record with tid >= 0 (no flag filtering, reference params.h:23-25 unused).
 * Reads of contig t are [tid_off[t], tid_off[t+1]) and are sorted by pos. */
typedef struct svt_pileup_view {
    int32_t         n_targets;
    const int64_t  *tid_off;    /* [n_targets+1]                                       */
    const int32_t  *pos;        /* [n_reads] bam1_core_t.pos (0-based)                  */
    const int32_t  *endpos;     /* [n_reads] htslib bam_endpos(): pos + max(1, rlen)    */
    const uint64_t *cig_off;    /* [n_reads+1] read r owns cigar[cig_off[r]..cig_off[r+1]) */
    const uint32_t *cigar;      /* BAM-packed ops, len << 4 | op                        */
    const uint8_t  *clip;       /* [n_reads] SVT_CLIP_* bits, or NULL: derive from cigar */
} svt_pileup_view;

/* Work counters of one batch (svt_count_work).  The first group is what the reference
 * algorithm touches (24 B/locus + 12 B/yielded read + 4 B/CIGAR word
 * walked); the others are what the engine's gather variant must read for the same batch --
 * its algorithmic bytes are `event_bytes` (DESIGN.md "Roofline"). */
typedef struct svt_work {
    uint64_t windows;        /* region queries issued (INV windows excluded)             */
    uint64_t reads;          /* reads yielded by the region queries                      */
    uint64_t ops_walked;     /* CIGAR words consumed by the walk loops, incl. the break op,
                                plus the soft-clip test word when not already walked      */
    uint64_t candidates;     /* breakpoint candidates pushed                              */
    uint64_t spilled_windows;/* windows whose candidates exceeded SVT_LDS_CANDS          */
    /* region query (event and span walks) + event walk (SVTREK_GATHER=event only) */
    uint64_t queries;        /* windows whose query reached the bucket table (32 B each)  */
    uint64_t probe_entries;  /* pos[]/emax[] entries the two searches need, boundary incl. */
    uint64_t range_reads;    /* reads in the query ranges [lo,hi): yielded (rec+rec2, 32 B)
                                plus overlap-failing ones (rec only, 16 B)                */
    uint64_t list_reads;     /* reads whose candidate-op list is read past the inline entry
                                (one 8-B list offset each)                                */
    uint64_t list_entries;   /* list entries read past the inline one (8 B each)          */
    uint64_t stop_searches;  /* refine_end break searches: 8 CIGAR words + 1 chunk word  */
    uint64_t stop_chunk_words; /* chunk-index words those searches scan, break chunk incl. */
    /* span walk (the default gather; zero for the others) */
    uint64_t span_bounds;    /* queries that read their span's two 8-B bounds             */
    uint64_t span_events;    /* 16-B events in the queries' spans                         */
    uint64_t event_bytes;    /* algorithmic bytes of the batch under the context's gather
                                variant: 24 B per locus + its reads at their byte sizes
                                (DESIGN.md "Roofline")                                    */
    /* value-bucketed event index (the default since 0.24; zero with SVTREK_INDEX=lists) */
    uint64_t bucket_queries; /* windows answered from the value buckets: two 4-B bucket
                                offsets + one 4-B prefix-max key each                      */
    uint64_t bucket_events;  /* 16-B events of the band's buckets, plus those of the
                                bounded walks for the facts above the band when the vote
                                needs them (event_bytes prices these instead of the span
                                walk's when the bucket index is on)                       */
} svt_work;

/* One refined call as the multi-GPU gather moves it: the record's index
 * in the VCF, its two results, padding.  index == 0xFFFFFFFF marks gather padding. */
typedef struct svt_record {
    uint32_t index;
    uint32_t start;
    uint32_t end;
    uint32_t pad;
} svt_record;

typedef struct svt_ctx svt_ctx;

/* Open a context on HIP device `device` (-1 = current).  Validates params. */
svt_status svt_open(const svt_params *params, int device, svt_ctx **out);

/* Open one context over `device_count` GPUs (devices[i], or 0 .. device_count-1 when
 * devices is NULL).  svt_load_pileup replicates the pileup on every device;
 * svt_refine_batch / svt_count_work / svt_sliding_window_ins split their batch into
 * contiguous slices, one per device, run concurrently and return results in input order.
 * The device-pointer calls (svt_refine_device*, svt_sync) and the POA mode act on the
 * first device.  device_count == 1 is svt_open(params, devices ? devices[0] : 0, out). */
svt_status svt_open_multi(const svt_params *params, int device_count, const int *devices, svt_ctx **out);
int        svt_device_count(const svt_ctx *ctx);

/* Copy the pileup to device HBM (replaces any previous one).  Synchronous. */
svt_status svt_load_pileup(svt_ctx *ctx, const svt_pileup_view *pileup);

/* Refine n host-resident loci into host-resident out[n].  Synchronous. */
svt_status svt_refine_batch(svt_ctx *ctx, const svt_locus *loci, size_t n, svt_result *out);

/* Refine n DEVICE-resident loci into DEVICE-resident out[n] on `hip_stream`
 * (a hipStream_t passed as void*, NULL = default stream).  Asynchronous: errors of
 * the launch itself are returned; spill-pool overflow is reported by svt_sync. */
svt_status svt_refine_device(svt_ctx *ctx, const svt_locus *d_loci, size_t n,
                             svt_result *d_out, void *hip_stream);

/* As svt_refine_device, but each result is written as a gather record
 * {d_index[i] (or index_base + i when d_index is NULL), start, end, 0}.
 * svt_reindex and the svt_refine_device* calls may be captured into a HIP graph (stream
 * capture on hip_stream, after one uncaptured call on that stream has sized the buffers):
 * every replay redoes the whole work, with the spill pool and left-over counters reset by the
 * graph itself.  A replay must not overlap other calls of the context. */
svt_status svt_refine_device_records(svt_ctx *ctx, const svt_locus *d_loci, size_t n,
                                     const uint32_t *d_index, uint32_t index_base,
                                     svt_record *d_rec, void *hip_stream);

/* Wait for `hip_stream` and report a deferred error (SVT_EOVERFLOW) of earlier calls.
 * On SVT_EOVERFLOW the context's spill pool has already been grown to what the failed
 * launch needed: re-running the same batch succeeds.  (svt_refine_batch and
 * svt_count_work do that re-run themselves.) */
svt_status svt_sync(svt_ctx *ctx, void *hip_stream);

/* Count the reference algorithm's work for n host loci (diagnostic, synchronous). */
svt_status svt_count_work(svt_ctx *ctx, const svt_locus *loci, size_t n, svt_work *out);

/* ---- optional mode: sliding_window_ins (reference sliding_window.c:8-97) ------------
 * Replaces int sliding_window_ins(int chrom, interval inter, t_arg *params, int
 * windowSize, int slideSize) (sliding_window.c:8; declared as refine_ins_disc in
 * sliding_window.h:11; the reference never calls it).  Query i covers the sub-windows
 * [s, min(s + window_size, end)) for s = start, start + window_size, ... < end; each is
 * refine_ins's region query and CIGAR walk, voted by sliding support (consensus_min_count
 * of the context's params).  best[i] = bestCandidateOverall (-1 = none).  If `sub` is not
 * NULL it receives, for every sub-window in query order, {bestCandidate, maxSupport}; the
 * reference prints "INS Discovery in window [%d, %d] at position %d with support %d\n"
 * for each sub-window whose bestCandidate != -1.  Synchronous.
 * EINVAL: window_size < 1 or slide_size < 1 (the reference loops forever), or
 * end + window_size > 2^32 (its uint32 sub_start wraps). */
typedef struct svt_sw_query { int32_t chrom; uint32_t start, end; } svt_sw_query;
typedef struct svt_sw_window { int32_t candidate, support; } svt_sw_window;

/* Sub-windows of one query: ceil((end - start) / window_size), 0 when end <= start. */
uint64_t   svt_sw_subwindows(const svt_sw_query *q, int32_t window_size);
svt_status svt_sliding_window_ins(svt_ctx *ctx, const svt_sw_query *q, size_t n, int32_t window_size,
                                  int32_t slide_size, int32_t *best, svt_sw_window *sub);

/* ---- optional mode: allele consensus of refined INS calls (POA) ----------------------
 * The north star's "abPOA banded partial-order consensus" step.  The reference declares
 * abPOA as a submodule (.gitmodules:4-6) but never includes or calls it (Makefile:16
 * links -lhts -lz -pthread only), so this mode has NO reference behaviour (parity
 * unpinned; its checker is oracle/poa_oracle.c) and never changes refined breakpoints.
 *
 * Sequences: the inserted bases of every I op with len >= 50 in the loaded pileup, in
 * (read, op) order of that pileup, as nt4 codes (0 A, 1 C, 2 G, 3 T, 4 other); sequence k
 * is bases[off[k] .. off[k+1]) and its length is the op's len.  For an INS call refined to
 * R, the supporting sequences are those I >= 50 ops of refine_ins's window reads
 * (refinement.c:290-316) processed by its walk, |position - R| <= support_radius and
 * len <= max_len, in read then op order; the first max_support are kept, the first
 * max_seqs that fit are fused (banded POA, w = band_b + band_f_permille * len / 1000), and
 * the heaviest bundle of the graph is the consensus. */
typedef struct svt_insseq_view {
    uint64_t        n_ins;   /* must equal svt_pileup_ins_count()                         */
    const uint64_t *off;     /* [n_ins + 1]                                               */
    const uint8_t  *bases;   /* [off[n_ins]] nt4 codes                                     */
} svt_insseq_view;

typedef struct svt_poa_params {
    int32_t match, mismatch, gap_open, gap_ext;  /* 2, 4, 4, 2 (a gap of L costs open + L*ext) */
    int32_t band_b, band_f_permille;             /* 10, 10; band_b + band_f * max_len / 1000 <= 63 */
    int32_t max_seqs, max_len, max_nodes;        /* 32 (<= 32), 4000 (<= 4096), 32768 (<= 65000) */
    int32_t support_radius, max_support;         /* 20, 64                                     */
} svt_poa_params;

typedef struct svt_poa_result {
    int32_t len;        /* consensus length (bases[0 .. min(len, cap)) written); -1: not a refined INS */
    int32_t n_support;  /* supporting sequences found                                     */
    int32_t n_used;     /* sequences fused into the graph                                 */
    int32_t status;     /* 0                                                              */
} svt_poa_result;

void       svt_poa_default_params(svt_poa_params *p);
/* I >= 50 ops in the loaded pileup (the length svt_load_insseq expects). */
uint64_t   svt_pileup_ins_count(const svt_ctx *ctx);
/* Copy the insertion sequences to the device (after svt_load_pileup).  Synchronous. */
svt_status svt_load_insseq(svt_ctx *ctx, const svt_insseq_view *seqs);
/* Consensus for n loci with their refined results (svt_refine_batch output): INS loci with a
 * refined start get a consensus in bases[i*cap ..], others len = -1.  Synchronous. */
svt_status svt_poa_consensus(svt_ctx *ctx, const svt_poa_params *p, const svt_locus *loci,
                             const svt_result *refined, size_t n, int32_t cap, uint8_t *bases,
                             svt_poa_result *res);
/* Loci the last svt_poa_consensus call reran on full-size scratch slots (their graphs
 * outgrew the small slots' node budget); a diagnostic, results do not depend on it. */
uint64_t   svt_poa_deferred(const svt_ctx *ctx);

/* Bytes of device memory the loaded pileup occupies. */
uint64_t svt_pileup_device_bytes(const svt_ctx *ctx);

/* Where the last svt_load_pileup spent its time.  The device index (per-read span-event
 * offsets and the span-event lists) depends only on the pileup, like the BAI the reference's
 * sam_itr_queryi needs (audit.c:271): it is the reference's per-read CIGAR walk
 * (refinement.c:118-159 / :184-221 / :295-318) done once per read instead of once per
 * (window, read). */
typedef struct svt_load_stats {
    double host_ms;      /* host pass: validation, prefix-max endpos, records, buckets, ranges  */
    double upload_ms;    /* synchronous H2D copies of the caller's arrays (CIGAR words incl.)    */
    double index_ms;     /* device index build (index_kind's kernels and their scans)            */
    double total_ms;     /* wall time of the whole svt_load_pileup call                          */
    uint64_t index_bytes;   /* algorithmic bytes one index build moves.  Lane per read (kind 1):
                               the CIGAR stream twice (4 B/op: census, emit), 65 B per read
                               (census: offsets + clip byte read, counts written; emit: counts,
                               offsets, record read, list offsets written), 16 B per span event
                               written.  Stream walk (kind 2): the stream once, 56 B per read
                               (offsets, records, staged and placed list offsets), 48 B per span
                               event (staged, read back, placed) */
    uint64_t span_events;   /* D-list + I-list span events of the pileup                         */
    uint64_t lead_blocks;   /* always 0 (the lead chunks of rounds 1-3 are gone since 0.17)      */
    uint64_t slow_reads;    /* reads whose walk reaches 2^28 bases or position 2^29              */
    uint64_t index_kind;    /* the index build used: 1 lane per read, 2 stream walk              */
    /* the value-bucketed event index (0.24, DESIGN.md "Value buckets"): every candidate event
     * filed by its candidate value in 1 kb buckets, per window kind -- the refine kernels read a
     * window's band from it, svt_reindex rebuilds it (and, with long reads, the span lists it is
     * filed from).  0 everywhere with SVTREK_INDEX=lists (the span lists alone, rounds 1-5). */
    uint64_t bucket_index;  /* 1: on                                                              */
    uint64_t buckets;       /* buckets per event array (every contig's, incl. its overflow bucket) */
    uint64_t bucket_events; /* events filed per rebuild (a D > 50 op twice: by start and by end)   */
    uint64_t bucket_bytes;  /* algorithmic bytes of one rebuild: lane per read, the CIGAR stream
                               once (4 B/op) + 24 B per read (offsets, record) + 28 B per filed
                               event (16-B event written, its bucket's two 4-B offsets read and
                               4-B cursor incremented); long reads (filed from the stream walk's
                               stage): the stream once + 32 B per read + 32 B per staged event
                               (written, read back) + 28 B per filed event                        */
} svt_load_stats;
svt_status svt_last_load_stats(const svt_ctx *ctx, svt_load_stats *out);

/* Rebuild the device index from the resident pileup on `hip_stream` (asynchronous, ordered
 * after every launch of the context already issued): the same two kernels svt_load_pileup
 * runs, no host work and no transfers.  Results of later refines are unchanged; bench.py
 * times it as part of every step so that the step covers the whole per-read walk. */
svt_status svt_reindex(svt_ctx *ctx, void *hip_stream);

/* ---- BGZF inflate (the BAM ingest's decompression on the device) ----
 * One BGZF block of a compressed buffer (SAM spec 4.1): its raw DEFLATE data comp[coff,
 * coff + clen) inflates to ulen bytes (the block's ISIZE) at out[uoff].  Replaces the inflate
 * behind htslib's bgzf_read, which the reference reaches through every sam_itr_next ->
 * bam_read1 (refinement.c:117, :186, :297). */
typedef struct svt_bgzf_block {
    uint64_t coff, uoff;
    uint32_t clen, ulen;
} svt_bgzf_block;
/* Inflate n blocks: comp (host, comp_bytes) -> out (host, out_bytes), synchronous.  Every
 * block must lie inside its buffers (<= 64 KiB each); SVT_EINVAL names the first block whose
 * data does not inflate to exactly ulen bytes. */
svt_status svt_bgzf_inflate(svt_ctx *ctx, const uint8_t *comp, size_t comp_bytes, const svt_bgzf_block *blocks,
                            size_t n, uint8_t *out, size_t out_bytes);
/* The same on device buffers (the block table on the device too; d_comp 16-B aligned and
 * readable up to 48 bytes past every block's data), asynchronous on hip_stream.  Calls of one
 * context share its scratch and error word, so they execute in submission order across streams
 * (as every launch of the context does).  svt_bgzf_inflate_status waits for the context's last
 * inflate (on hip_stream, ordered after it) and reports its first corrupt block (0xffffffff: none). */
svt_status svt_bgzf_inflate_device(svt_ctx *ctx, const uint8_t *d_comp, const svt_bgzf_block *d_blocks, size_t n,
                                   uint8_t *d_out, void *hip_stream);
svt_status svt_bgzf_inflate_status(svt_ctx *ctx, void *hip_stream, uint32_t *bad_block);
/* Device time (ms, HIP events) of the last svt_bgzf_inflate's kernel. */
double svt_bgzf_last_inflate_ms(const svt_ctx *ctx);
/* Pinned host memory on the context's device (svt_bgzf_inflate copies from / to it at full
 * PCIe speed); NULL on failure.  Free with svt_host_free. */
void *svt_host_alloc(svt_ctx *ctx, size_t bytes);
void  svt_host_free(svt_ctx *ctx, void *p);

/* ---- BAM records decoded on the device ---------------------------------
 * Replaces, for this path, htslib's bam_read1 behind every sam_itr_next (reference
 * refinement.c:117; the path reads core.tid/pos/flag/n_cigar and the CIGAR, :118-120) and the
 * host ingest's record parse: the BAM's BGZF blocks go to the device compressed, are inflated
 * there, and their records are found, parsed (CG:B,I CIGARs restored as htslib's bam_tag2cigar
 * does) and appended to a device-resident columnar pileup -- no inflated byte crosses PCIe.
 * Records with tid < 0 / tid >= n_targets / pos < 0 are skipped (no tid >= 0 query yields them).
 *   svt_bam_dec_open:  a decoder on ctx's device for a BAM with n_targets references;
 *   svt_bam_dec_feed:  the next batch of whole BGZF blocks of the file, in order (host buffers,
 *                      the layout of svt_bgzf_inflate, uoff relative to the batch); the first
 *                      `skip` inflated bytes of the first batch are the BAM header (not records);
 *                      a record may span batches.  Pipelined one batch deep: the call returns
 *                      once its batch's bytes are on the device and its inflate is launched, and
 *                      that batch is decoded by the next call or by svt_bam_dec_load (so a
 *                      corrupt block or record may be reported there); the host buffers may be
 *                      reused as soon as the call returns.
 *   svt_bam_dec_load:  at the end of the file: the decoded pileup becomes ctx's pileup, exactly
 *                      as svt_load_pileup of the same reads (a file not sorted by coordinate is
 *                      sorted, as the host ingest does); SVT_EINVAL for a truncated last record.
 * Errors: SVT_EINVAL for a corrupt BGZF block or BAM record (message in svt_last_error(ctx)). */
typedef struct svt_bam_dec svt_bam_dec;
typedef struct svt_bam_dec_stats {
    uint64_t records;         /* complete records decoded (all tids)                          */
    uint64_t reads;           /* records kept for the pileup                                  */
    uint64_t cigar_ops;       /* their CIGAR ops (after CG restoration)                        */
    uint64_t cg_restored;     /* CIGARs restored from a CG:B,I tag                             */
    uint64_t batches;         /* svt_bam_dec_feed calls                                       */
    uint64_t rechained;       /* batches whose record starts were re-chained hop by hop        */
    uint64_t inflated_bytes;  /* bytes the batches inflated to                                 */
    double   feed_ms;         /* wall time inside svt_bam_dec_feed (H2D, inflate, decode)       */
    uint64_t rechained_chunks;/* 64 KiB chunks those re-chains walked (from the first wrong guess) */
} svt_bam_dec_stats;
svt_status svt_bam_dec_open(svt_ctx *ctx, int32_t n_targets, svt_bam_dec **out);
svt_status svt_bam_dec_feed(svt_bam_dec *dec, const uint8_t *comp, size_t comp_bytes, const svt_bgzf_block *blocks,
                            size_t n, uint64_t skip);
svt_status svt_bam_dec_load(svt_bam_dec *dec);
svt_status svt_bam_dec_stats_get(const svt_bam_dec *dec, svt_bam_dec_stats *out);
void       svt_bam_dec_close(svt_bam_dec *dec);

const char *svt_last_error(const svt_ctx *ctx);
void        svt_close(svt_ctx *ctx);
const char *svt_version(void);

/* LDS candidate capacity per window; larger windows spill to the device pool. */
#define SVT_LDS_CANDS 256

#ifdef __cplusplus
}
#endif
#endif /* SVTREK_GPU_H */
