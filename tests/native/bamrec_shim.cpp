// Test shim: svt_bamrec.h's record-start guess compiled for the host (tests/test_bam_decode.py).
#include "svt_bamrec.h"

extern "C" uint64_t bamrec_scan(const uint8_t *buf, uint64_t n, int32_t n_ref, uint64_t *out, uint64_t cap) {
    uint64_t k = 0;
    for (uint64_t p = 0; p < n && k < cap; p++)
        if (bamrec::plausible(buf, p, n, n_ref)) out[k++] = p;
    return k;
}
