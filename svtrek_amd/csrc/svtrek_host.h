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
void      svth_bam_free(svth_bam *b);
/* View valid until svth_bam_free. */
void      svth_bam_view(const svth_bam *b, svt_pileup_view *out);
int32_t   svth_bam_n_targets(const svth_bam *b);
const char *svth_bam_target_name(const svth_bam *b, int32_t tid);
int64_t   svth_bam_n_records(const svth_bam *b);     /* all records incl. tid < 0     */
int64_t   svth_bam_n_cg_restored(const svth_bam *b); /* CIGARs restored from CG:B,I   */

/* A1: parse one VCF data line in place (as strtok_r does).
 * Returns 1 = record reaches the type switch (*l filled), 0 = skipped silently,
 * 2 = skipped with a stderr message (written into err). */
int svth_parse_line(char *line, svt_locus *l, char *err, size_t errcap);

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
