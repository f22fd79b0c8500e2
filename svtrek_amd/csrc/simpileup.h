/*
 * simpileup.h -- seeded synthetic long-read pileups for the audt path (test/bench data).
 *
 * The reference never reads SEQ/QUAL on this path (refinement.c:118-120 uses only
 * core.pos, n_cigar and the CIGAR), so a pileup is generated directly as alignments:
 * read start + CIGAR, no aligner.  SV loci carry breakpoint evidence the way
 * SURVEY.md §8(d) describes: reads spanning a DEL carry a D op (or are split with a
 * trailing S + a supplementary with a leading H/S), reads spanning an INS carry an I op,
 * with per-read breakpoint jitter; noise ops model ONT/HiFi error profiles.
 */
#ifndef SVTREK_SIMPILEUP_H
#define SVTREK_SIMPILEUP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct sim_config {
    uint64_t seed;
    int32_t  n_targets;        /* contigs "1".."n" (tid 0..n-1)                          */
    int32_t  n_loci;           /* SV loci, spread evenly over the contigs                */
    double   del_frac;         /* fraction DEL (rest INS)                                */
    int32_t  sv_min_len, sv_max_len;   /* log-uniform SV length                         */
    int32_t  spacing;          /* locus spacing along a contig (>= 30 kb keeps windows apart) */
    int32_t  first_offset;     /* first locus at >= this position (avoid window wrap)    */
    double   coverage;         /* mean depth                                             */
    int32_t  read_len_mean, read_len_sd, read_len_min;
    double   rho;              /* CIGAR ops per reference bp (SURVEY §8 notation)        */
    double   p_carry;          /* spanning read carries the SV op                        */
    double   p_split;          /* spanning read is split at a DEL (trailing S + supplementary) */
    int32_t  bp_jitter;        /* per-read breakpoint jitter, uniform [-j, j]            */
    int32_t  report_jitter;    /* VCF pos/end offset from the true breakpoint, [-r, r]   */
    double   p_noise_sv;       /* per read: one unrelated D/I >= 50 bp                   */
    double   p_clip_ends;      /* per read end: short soft clip / hard clip              */
    double   p_exotic;         /* per error op: N, H, P or a code 9..15 op (quirk coverage) */
    int32_t  par_contigs;      /* != 0: each contig's reads from its own PRNG stream, one thread
                                  per contig (a different, equally seeded pileup; 0: one stream) */
} sim_config;

typedef struct sim_pileup sim_pileup;

/* Generate; returns NULL on allocation failure. */
sim_pileup *sim_generate(const sim_config *cfg);
void        sim_free(sim_pileup *p);

/* Columnar views (owned by the sim_pileup, valid until sim_free). */
int32_t         sim_n_targets(const sim_pileup *p);
int32_t         sim_contig_len(const sim_pileup *p, int32_t tid);
int64_t         sim_n_reads(const sim_pileup *p);
uint64_t        sim_n_ops(const sim_pileup *p);
const int64_t  *sim_tid_off(const sim_pileup *p);
const int32_t  *sim_pos(const sim_pileup *p);
const int32_t  *sim_endpos(const sim_pileup *p);
const uint64_t *sim_cig_off(const sim_pileup *p);
const uint32_t *sim_cigar(const sim_pileup *p);
const uint16_t *sim_flag(const sim_pileup *p);
int32_t         sim_n_loci(const sim_pileup *p);
/* loci as {type, chrom, pos, end} (reported, jittered) + true breakpoints */
const int32_t  *sim_loci(const sim_pileup *p);        /* [n_loci*4]                        */
const int32_t  *sim_truth(const sim_pileup *p);       /* [n_loci*2] true bp1, bp2          */

/* Insertion sequences for the allele-consensus mode: for every I op with len >= 50, in
 * (read, op) order, `len` nt4 bases (0 A, 1 C, 2 G, 3 T).  An I op carrying an INS locus's
 * allele (an INS locus of the read's contig whose true bp1 is within bp_jitter + 1 of the
 * op's walk position and whose length equals the op's) gets that locus's allele (random,
 * seeded per locus) with per-base substitutions at err_permille / 1000; any other I op gets
 * random bases.  *off ([n+1]) and *bases are malloc'ed (free with sim_free_buf).  0 / -1. */
int  sim_insseq(const sim_pileup *p, uint64_t seed, int32_t bp_jitter, int32_t err_permille, uint64_t *n_ins,
                uint64_t **off, uint8_t **bases);
void sim_free_buf(void *x);

/* Write the pileup as a BGZF-compressed, coordinate-sorted BAM.  with_seq != 0 stores
 * random SEQ/QUAL of the CIGAR's query length (realistic ingest cost).  0 on success. */
int sim_write_bam(const sim_pileup *p, const char *path, int with_seq, int level);
/* The same, restricted to the records of contig `tid` overlapping [beg, end) (tid < 0: all
 * records), and with write_bai != 0 also `path`.bai: bins + chunks + the 16 kb linear index
 * (SAM spec 5.2; empty windows hold the next window's offset).  0 on success. */
int sim_write_bam_region(const sim_pileup *p, const char *path, int with_seq, int level, int32_t tid, int64_t beg,
                         int64_t end, int write_bai);
/* the records overlapping any of nreg regions (tid[k], [beg[k], end[k])) -- a shard's halo of
 * several contigs; nreg == 0: every record */
int sim_write_bam_regions(const sim_pileup *p, const char *path, int with_seq, int level, int nreg, const int32_t *tid,
                          const int64_t *beg, const int64_t *end, int write_bai);

#ifdef __cplusplus
}
#endif
#endif
