// svt_bamrec.h -- one BAM record (SAM spec 4.2) as the audt path reads it: the fields
// htslib's bam_read1 decodes that refinement.c:117-120 uses (core.tid/pos/flag/n_cigar and the
// CIGAR, restored from a CG:B,I tag as bam_tag2cigar does) and the two soft-clip test words
// the reference reads.  Host and device code share it: the host ingest (bam_ingest.cpp) and
// the device record decode (svt_bam.inc) read records through these functions.
//
// Everything reads bytes (records sit at any byte offset of an inflated BAM stream).
#ifndef SVT_BAMREC_H
#define SVT_BAMREC_H

#include <stddef.h>
#include <stdint.h>

#ifndef SVT_HD
#if defined(__HIPCC__)
#define SVT_HD __host__ __device__ __forceinline__
#else
#define SVT_HD inline
#endif
#endif

namespace bamrec {

constexpr uint32_t OP_M = 0, OP_D = 2, OP_N = 3, OP_S = 4, OP_EQ = 7, OP_X = 8;
constexpr uint32_t CLIP_LAST_S = 0x1u, CLIP_FIRST_S = 0x2u;   // = SVT_CLIP_LAST_S / SVT_CLIP_FIRST_S

SVT_HD uint32_t rd16(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8; }
SVT_HD uint32_t rd32(const uint8_t *p) {
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

// Where a record's CIGAR lives (after CG restoration) and its soft-clip test bits.  `r` is the
// record after its block_size word, `bs` that block_size.
struct View {
    const uint8_t *cig;   // n words (unaligned)
    uint32_t n;
    bool cg;              // restored from CG:B,I
    bool ok;              // tid >= 0 && tid < n_ref && pos >= 0: a record a region query can yield
    bool bad;             // ok but its CIGAR / SEQ run past the record: a corrupt file
    int32_t tid, pos;
    uint32_t flag;
    uint32_t clip;
};

// htslib bam_tag2cigar's conditions: n_cigar > 0, tid >= 0, pos >= 0, cigar[0] == <l_seq>S,
// a CG tag of type B,I (or B,i) with at least n_cigar elements and fewer than 2^29.
SVT_HD bool find_cg(const uint8_t *aux, const uint8_t *end, const uint8_t **arr, uint32_t *cnt) {
    const uint8_t *p = aux;
    while (p + 3 <= end) {
        const char t0 = (char)p[0], t1 = (char)p[1], ty = (char)p[2];
        p += 3;
        size_t sz = 0;
        switch (ty) {
        case 'A': case 'c': case 'C': sz = 1; break;
        case 's': case 'S': sz = 2; break;
        case 'i': case 'I': case 'f': sz = 4; break;
        case 'Z': case 'H': {
            const uint8_t *q = p;
            while (q < end && *q) q++;
            if (q >= end) return false;
            p = q + 1;
            continue;
        }
        case 'B': {
            if (p + 5 > end) return false;
            const char sub = (char)p[0];
            const uint32_t n = rd32(p + 1);
            const size_t es = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2
                              : (sub == 'i' || sub == 'I' || sub == 'f') ? 4 : 0;
            if (!es) return false;
            if (t0 == 'C' && t1 == 'G') {
                if (sub != 'I' && sub != 'i') return false;
                if (p + 5 + (size_t)n * 4 > end) return false;
                *arr = p + 5;
                *cnt = n;
                return true;
            }
            p += 5 + (size_t)n * es;
            continue;
        }
        default:
            return false;
        }
        p += sz;
    }
    return false;
}

SVT_HD View view(const uint8_t *r, uint32_t bs, int32_t n_ref) {
    View v{};
    const uint8_t *rend = r + bs;
    v.tid = (int32_t)rd32(r);
    v.pos = (int32_t)rd32(r + 4);
    const uint32_t l_qname = r[8];
    const uint32_t n_cig = rd16(r + 12);
    v.flag = rd16(r + 14);
    const int32_t l_seq = (int32_t)rd32(r + 16);
    v.ok = v.tid >= 0 && v.tid < n_ref && v.pos >= 0;   // only these can be yielded by a tid >= 0 query
    if (!v.ok) return v;
    const uint8_t *qn = r + 32, *cg = qn + l_qname;
    if (cg + 4ull * n_cig > rend || l_seq < 0) { v.bad = true; return v; }
    const uint8_t *after = cg + 4ull * n_cig;   // SEQ starts here
    const uint8_t *aux = after + (size_t)(l_seq + 1) / 2 + (size_t)l_seq;
    v.cig = cg;
    v.n = n_cig;
    if (n_cig > 0 && (rd32(cg) & 0xfu) == OP_S && (int64_t)(rd32(cg) >> 4) == l_seq && aux <= rend) {
        const uint8_t *arr;
        uint32_t cnt;
        if (find_cg(aux, rend, &arr, &cnt) && cnt >= n_cig && cnt < (1u << 29)) { v.cig = arr; v.n = cnt; v.cg = true; }
    }
    // Soft-clip test words as the reference reads them through bam1_t.data: the qname is
    // padded with NULs to a multiple of 4 (htslib l_extranul), so cigar[-1] is the last 4
    // bytes of the padded name and cigar[0] of an empty CIGAR is the first SEQ byte.
    uint32_t c = 0;
    if (v.n) {
        if ((rd32(v.cig + 4ull * (v.n - 1)) & 0xfu) == OP_S) c |= CLIP_LAST_S;
        if ((rd32(v.cig) & 0xfu) == OP_S) c |= CLIP_FIRST_S;
    } else {
        const uint32_t padded = (l_qname + 3u) & ~3u;
        const uint8_t lastw0 = (padded >= 4 && padded - 4 < l_qname) ? qn[padded - 4] : 0;
        if ((lastw0 & 0xfu) == OP_S) c |= CLIP_LAST_S;
        if (after < rend && (after[0] & 0xfu) == OP_S) c |= CLIP_FIRST_S;
    }
    v.clip = c;
    return v;
}

// htslib bam_endpos: pos + the reference length of the CIGAR (M/D/N/=/X), or pos + 1 when the
// read is unmapped (flag 4) or its CIGAR consumes no reference.
SVT_HD int32_t endpos(const View &v) {
    int64_t rl = 0;
    if (!(v.flag & 4))
        for (uint32_t j = 0; j < v.n; j++) {
            const uint32_t w = rd32(v.cig + 4ull * j), op = w & 0xfu;
            if (op == OP_M || op == OP_D || op == OP_N || op == OP_EQ || op == OP_X) rl += w >> 4;
        }
    return (int32_t)(v.pos + (rl ? rl : 1));
}

// Could a record start at p (its block_size word) of the bytes [buf, buf + n)?  Necessary
// conditions of every well-formed record (SAM spec 4.2): refID and next_refID in [-1, n_ref),
// pos and next_pos >= -1, l_read_name >= 1, l_seq >= 0, the fixed fields, name, CIGAR, SEQ and
// QUAL inside block_size, a NUL-terminated name without other NULs.  The device decode guesses
// record starts with it and then proves the guesses on the chain of block_size hops, so a
// false guess costs time, never a wrong result.
SVT_HD bool plausible(const uint8_t *buf, uint64_t p, uint64_t n, int32_t n_ref) {
    if (p + 36 > n) return false;
    const uint8_t *r = buf + p + 4;
    const uint32_t bs = rd32(buf + p);
    const int32_t tid = (int32_t)rd32(r), pos = (int32_t)rd32(r + 4);
    if (bs < 32 || tid < -1 || tid >= n_ref || pos < -1) return false;
    const int32_t ntid = (int32_t)rd32(r + 20), npos = (int32_t)rd32(r + 24);
    if (ntid < -1 || ntid >= n_ref || npos < -1) return false;
    const uint32_t l_qname = r[8], n_cig = rd16(r + 12);
    const int32_t l_seq = (int32_t)rd32(r + 16);
    if (l_qname < 1 || l_seq < 0) return false;
    if (32ull + l_qname + 4ull * n_cig + (uint64_t)(l_seq + 1) / 2 + (uint64_t)l_seq > bs) return false;
    if (p + 36 + l_qname > n) return false;
    const uint8_t *qn = r + 32;
    if (qn[l_qname - 1] != 0) return false;
    for (uint32_t i = 0; i + 1 < l_qname; i++)
        if (qn[i] == 0) return false;
    return true;
}

}  // namespace bamrec

#endif
