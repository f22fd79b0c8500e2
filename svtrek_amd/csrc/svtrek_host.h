/*
 * svtrek_host.h -- host side of the `svtrek audt` drop-in (C ABI, plain types).
 *
 *  - BAM/BGZF ingest -> columnar pileup (replaces, for this path, htslib's
 *    hts_open/sam_hdr_read/sam_index_load + the per-window sam_itr_queryi/sam_itr_next
 *    decode of reference refinement.c:114-117; the whole file is read once, multi-
 *    threaded inflate, SEQ/QUAL/aux dropped except the CG tag).
 *  - VCF record parsing (A1, reference audit.c:62-173) and result printing (A11,
 *    audit.c:176-232), byte-identical to the reference's stdout.
 */
#ifndef SVTREK_HOST_H
#define SVTREK_HOST_H

#include <stddef.h>
#include <stdint.h>

#include "svtrek_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct svth_bam svth_bam;

/* Read a BAM (BGZF) completely into a columnar pileup.  threads >= 1 inflate workers.
 * Returns NULL on error (message in err). */
svth_bam *svth_bam_read(const char *path, int threads, char *err, size_t errcap);
/* The records of a coordinate-sorted BAM from (tid0, beg0) up to, excluding, the first
 * record at or past (tid1, end1), read from the BAI's linear-index offset of (tid0, beg0)
 * (`path`.bai, required; the file's header is read from its start).  Every region query
 * (tid, [beg, end)) with (tid0, beg0) <= (tid, beg) and (tid, end) <= (tid1, end1) yields the
 * same reads from this pileup as from the whole file; a few records before beg0 may be
 * included.  tid0 < 0: the whole file (svth_bam_read). */
svth_bam *svth_bam_read_region(const char *path, int threads, int32_t tid0, int64_t beg0, int32_t tid1, int64_t end1,
                               char *err, size_t errcap);
/* A BGZF inflater for the ingest (svth_bam_read_ex): inflate(n blocks of comp -> out, the
 * layout of svt_bgzf_inflate, include/svtrek_gpu.h; 0 = done, else a message in err); alloc /
 * release (optional): the buffers inflate reads and writes fastest (pinned host memory);
 * batch_bytes: compressed bytes per inflate call (0: 1 GiB). */
typedef struct svth_inflater {
    int (*inflate)(void *user, const uint8_t *comp, size_t comp_bytes, const svt_bgzf_block *blocks, size_t n,
                   uint8_t *out, size_t out_bytes, char *err, size_t errcap);
    void *(*alloc)(void *user, size_t bytes);
    void (*release)(void *user, void *p);
    void *user;
    size_t batch_bytes;
} svth_inflater;
/* svth_bam_read_region with the BGZF blocks inflated by `inf` (the CLI passes the device's
 * svt_bgzf_inflate and pinned buffers): batches read by `threads` parallel preads, the next
 * batch read and inflated by a helper thread while the records of the current one are parsed;
 * inf == NULL: host threads inflate. */
svth_bam *svth_bam_read_ex(const char *path, int threads, int32_t tid0, int64_t beg0, int32_t tid1, int64_t end1,
                           const svth_inflater *inf, char *err, size_t errcap);
/* A BAM decoded on the device: the file read in batches of whole BGZF blocks (`threads`
 * parallel preads; buffers from sink->alloc when given, e.g. pinned memory) and handed to
 * sink->feed compressed -- the next batch read by a helper thread meanwhile.  The header is
 * inflated and read on the host: sink->begin gets its reference count first, and the first
 * feed's `skip` is its length in the inflated stream (the CLI's sink is svt_bam_dec_*).
 * stage4 (optional): batch reads, feed calls, waits for the next batch, the whole read (s).
 * Returns 0, or 1 with a message in err. */
typedef struct svth_dev_sink {
    int (*begin)(void *user, int32_t n_targets, char *err, size_t errcap);
    int (*feed)(void *user, const uint8_t *comp, size_t comp_bytes, const svt_bgzf_block *blocks, size_t n,
                uint64_t skip, char *err, size_t errcap);
    void *(*alloc)(void *user, size_t bytes);
    void (*release)(void *user, void *p);
    void *user;
    size_t batch_bytes;   /* compressed bytes per batch (0: 1 GiB) */
} svth_dev_sink;
int svth_bam_read_device(const char *path, int threads, const svth_dev_sink *sink, int32_t *n_targets, double *stage4,
                         char *err, size_t errcap);
void      svth_bam_free(svth_bam *b);
/* View valid until svth_bam_free. */
void      svth_bam_view(const svth_bam *b, svt_pileup_view *out);
int32_t   svth_bam_n_targets(const svth_bam *b);
const char *svth_bam_target_name(const svth_bam *b, int32_t tid);
int64_t   svth_bam_n_records(const svth_bam *b);     /* all records incl. tid < 0     */
int64_t   svth_bam_n_cg_restored(const svth_bam *b); /* CIGARs restored from CG:B,I   */
/* Where a device-inflate read spent its time (s): batch reads, header scans, buffer allocation,
 * inflate calls (all on the helper thread), the parser waiting for batches, and the whole read. */
void      svth_bam_stage_seconds(const svth_bam *b, double *s6);

/* A1: parse one VCF data line in place (as strtok_r does).
 * Returns 1 = record reaches the type switch (*l filled), 0 = skipped silently,
 * 2 = skipped with a stderr message (written into err). */
int svth_parse_line(char *line, svt_locus *l, char *err, size_t errcap);

/* A1 over a whole VCF text (the reader loop of process_vcf, audit.c:295-338: lines shorter
 * than 2 bytes and '#' lines skipped, the trailing '\n' stripped), parsed by `threads`
 * threads over '\n'-aligned pieces.  Records in file order; the stderr messages the
 * reference's workers would print (parse errors, "[ERROR] Unkown type.") in file order. */
typedef struct svth_vcf svth_vcf;
svth_vcf        *svth_vcf_parse(const char *text, size_t len, int threads);
size_t           svth_vcf_count(const svth_vcf *v);
const svt_locus *svth_vcf_loci(const svth_vcf *v);
const char      *svth_vcf_messages(const svth_vcf *v, size_t *len);
void             svth_vcf_free(svth_vcf *v);

/* A11 over a batch: the concatenated stdout text of n records in order, formatted by
 * `threads` threads; malloc'ed (free with svth_free), *len = its length. */
char *svth_format_batch(const svt_locus *l, const svt_result *r, size_t n, int threads, size_t *len);
void  svth_free(void *p);

/* A11: stdout text for one refined record; returns bytes written (0 = prints nothing:
 * DUP/TRA/BND/unknown -> "[ERROR] Unkown type." on stderr, or DEL/INV of exactly 50 bp). */
int svth_format(const svt_locus *l, const svt_result *r, char *buf, size_t cap);
/* 1 when the record's type has no refinement (the reference prints
 * "[ERROR] Unkown type.\n" to stderr for it, audit.c:233-235). */
int svth_is_unknown_type(const svt_locus *l);

#ifdef __cplusplus
}
#endif
#endif
