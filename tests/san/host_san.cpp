// Sanitizer driver for the product's host C++ (bam_ingest.cpp, vcf_audit.cpp): built with
// ASan+UBSan or TSan by tests/test_sanitizers.py, run on test BAMs / VCFs.  Prints one
// line of checksums that the test compares with the uninstrumented library's results.
//   host_san BAM VCF THREADS [tid0 beg0 tid1 end1]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "svtrek_host.h"

static uint64_t mix(uint64_t h, uint64_t v) { return (h ^ v) * 0x100000001b3ull; }

int main(int argc, char **argv) {
    if (argc < 4) return 2;
    const int T = atoi(argv[3]);
    char err[512];
    svth_bam *b = argc >= 8 ? svth_bam_read_region(argv[1], T, atoi(argv[4]), atoll(argv[5]), atoi(argv[6]),
                                                   atoll(argv[7]), err, sizeof err)
                            : svth_bam_read(argv[1], T, err, sizeof err);
    if (!b) { fprintf(stderr, "bam: %s\n", err); return 1; }
    svt_pileup_view v;
    svth_bam_view(b, &v);
    const int64_t n = v.tid_off[v.n_targets];
    uint64_t h = 0xcbf29ce484222325ull;
    for (int64_t r = 0; r < n; r++) {
        h = mix(h, (uint32_t)v.pos[r]);
        h = mix(h, (uint32_t)v.endpos[r]);
        h = mix(h, v.clip ? v.clip[r] : 0);
        for (uint64_t k = v.cig_off[r]; k < v.cig_off[r + 1]; k++) h = mix(h, v.cigar[k]);
    }
    printf("reads %lld records %lld cg %lld bamsum %016llx", (long long)n, (long long)svth_bam_n_records(b),
           (long long)svth_bam_n_cg_restored(b), (unsigned long long)h);
    svth_bam_free(b);

    FILE *f = fopen(argv[2], "rb");
    if (!f) return 1;
    std::string text;
    char buf[1 << 16];
    size_t k;
    while ((k = fread(buf, 1, sizeof buf, f)) > 0) text.append(buf, k);
    fclose(f);
    svth_vcf *pv = svth_vcf_parse(text.data(), text.size(), T);
    const size_t m = svth_vcf_count(pv);
    const svt_locus *l = svth_vcf_loci(pv);
    svt_result *res = (svt_result *)malloc(sizeof(svt_result) * (m ? m : 1));
    uint64_t lh = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < m; i++) {
        lh = mix(mix(mix(mix(lh, (uint32_t)l[i].type), (uint32_t)l[i].chrom), l[i].pos), l[i].end);
        res[i].start = (i % 3 == 0) ? SVT_NA : l[i].pos + (uint32_t)(i % 7) - 3u;
        res[i].end = (i % 5 == 0) ? SVT_NA : l[i].end - (uint32_t)(i % 11);
    }
    size_t ml = 0;
    svth_vcf_messages(pv, &ml);
    size_t ol = 0;
    char *out = svth_format_batch(l, res, m, T, &ol);
    uint64_t oh = 0xcbf29ce484222325ull;
    for (size_t i = 0; i < ol; i++) oh = mix(oh, (uint8_t)out[i]);
    printf(" loci %zu locisum %016llx msgbytes %zu outbytes %zu outsum %016llx\n", m, (unsigned long long)lh, ml, ol,
           (unsigned long long)oh);
    svth_free(out);
    free(res);
    svth_vcf_free(pv);
    return 0;
}
