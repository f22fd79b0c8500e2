/* Sanitizer driver for the oracle's threaded paths (test infrastructure): the pthread batch
 * over the in-memory pileup and the BGZF baseline's per-thread readers, on a generated
 * pileup and BAM (+ BAI) -- results must agree.  Built with ASan+UBSan or TSan by
 * tests/test_sanitizers.py.   oracle_san DIR THREADS */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "simpileup.h"
#include "svtrek_oracle.h"

int main(int argc, char **argv) {
    if (argc < 3) return 2;
    const int T = atoi(argv[2]);
    sim_config c;
    memset(&c, 0, sizeof c);
    c.seed = 77; c.n_targets = 2; c.n_loci = 150; c.del_frac = 0.5; c.sv_min_len = 50; c.sv_max_len = 2000;
    c.spacing = 40000; c.first_offset = 25000; c.coverage = 10.0; c.read_len_mean = 8000; c.read_len_sd = 2000;
    c.read_len_min = 1000; c.rho = 1.0 / 40; c.p_carry = 0.7; c.p_split = 0.15; c.bp_jitter = 8;
    c.report_jitter = 40; c.p_noise_sv = 0.05; c.p_clip_ends = 0.2; c.p_exotic = 0.01;
    sim_pileup *p = sim_generate(&c);
    if (!p) return 1;
    char bam[4096];
    snprintf(bam, sizeof bam, "%s/o.bam", argv[1]);
    if (sim_write_bam_region(p, bam, 1, 1, -1, 0, 0, 1)) return 1;
    orc_pileup v = {sim_n_targets(p), sim_tid_off(p), sim_pos(p), sim_endpos(p), sim_cig_off(p), sim_cigar(p), NULL};
    const int32_t n = sim_n_loci(p);
    const int32_t *L = sim_loci(p);
    orc_locus *loci = (orc_locus *)malloc(sizeof(orc_locus) * (size_t)n);
    for (int32_t i = 0; i < n; i++) {
        loci[i].type = L[4 * i]; loci[i].chrom = L[4 * i + 1];
        loci[i].pos = (uint32_t)L[4 * i + 2]; loci[i].end = (uint32_t)L[4 * i + 3];
    }
    orc_params prm = {20000, 10000, 2000, 500, 5, 3};
    orc_result *a = (orc_result *)malloc(sizeof(orc_result) * (size_t)n);
    orc_result *b = (orc_result *)malloc(sizeof(orc_result) * (size_t)n);
    orc_work w;
    if (orc_refine_batch(&v, &prm, loci, (size_t)n, a, T, &w)) return 1;
    uint64_t st[3];
    char err[256];
    if (orc_bgzf_refine_batch(bam, &prm, loci, (size_t)n, b, T, st, err, sizeof err)) { fprintf(stderr, "%s\n", err); return 1; }
    int same = memcmp(a, b, sizeof(orc_result) * (size_t)n) == 0;
    int refined = 0;
    for (int32_t i = 0; i < n; i++) refined += a[i].start != 0xFFFFFFFFu;
    printf("loci %d refined %d same %d blocks %llu\n", n, refined, same, (unsigned long long)st[0]);
    free(a); free(b); free(loci);
    sim_free(p);
    return same ? 0 : 1;
}
