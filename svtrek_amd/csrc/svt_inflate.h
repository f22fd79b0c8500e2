// svt_inflate.h -- raw DEFLATE (RFC 1951) decoder for one BGZF block, written once for the
// host compiler (tests against zlib) and the gfx950 device (one lane per block).
//
// What the reference gets from htslib's bgzf_read (refinement.c:117 sam_itr_next ->
// bam_read1 -> bgzf_read -> inflate) is the block's bytes; this decodes the same bytes.
// Lane-serial by design: DEFLATE is a serial bitstream, and a BAM has one independent block
// per <= 64 KiB of output, so a batch of blocks is one lane each.
//
//   * litlen / dist codes: a primary table of IF_LB / IF_DB bits (bit-reversed index, as the
//     stream is LSB-first), entry = symbol | length << 9; codes longer than the table take the
//     canonical slow path (per-length counts + symbols sorted by code, RFC 1951 3.2.2)
//   * the primary tables live in the caller's fast memory (LDS on the device), the slow-path
//     arrays and code lengths in a per-lane scratch area (global memory on the device)
//   * every input read is bounds-checked against the block's compressed length (reads past it
//     see zeros and fail the block), every output write against its ISIZE
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define SVT_HD __host__ __device__ __forceinline__
#else
#define SVT_HD inline
#endif

#ifndef SVT_IF_LB
#define SVT_IF_LB 8
#endif
#ifndef SVT_IF_DB
#define SVT_IF_DB 6
#endif
constexpr int IF_LB = SVT_IF_LB;   // litlen primary table bits (256 entries)
constexpr int IF_DB = SVT_IF_DB;   // dist primary table bits (64 entries)

// The primary tables of one block, `stride` entries apart (the device interleaves the 64 lanes'
// tables in LDS, lane-minor, so that any mix of indices is bank-conflict free): 640 B a block.
constexpr int IF_FAST = (1 << IF_LB) + (1 << IF_DB);
struct InfTab {
    uint16_t *p;
    int stride;
    SVT_HD uint16_t &operator[](int i) const { return p[i * stride]; }
};
struct InfFast {
    InfTab lit, dst;
    SVT_HD InfFast(uint16_t *base, int stride) : lit{base, stride}, dst{base + (1 << IF_LB) * stride, stride} {}
};
struct InfSlow {               // per block, scratch
    uint16_t lcnt[16], dcnt[16], offs[16];
    uint16_t lsym[288], dsym[32];
    uint8_t len[320];          // code lengths being read (litlen, then dist from 288 on)
    uint8_t cl[20];            // code-length code lengths
};

enum : int { INF_OK = 0, INF_EDATA = 1, INF_EOUT = 2, INF_EIN = 3 };

// The bit reader takes the stream as 16-B aligned vectors: the block's data starts `skip` bytes
// (< 16) into vector 0, and vectors past the last one holding data read as zeros (a valid stream
// never consumes them; past() tells a stream that did).  Two vectors beyond the one being
// consumed are always in flight (a lane's next loads are issued ~ 32 bytes before their bits
// are needed, so the decode does not wait on them).  fill() leaves >= 33 bits buffered, which
// covers every step between two fills (a code of <= 15 bits + <= 13 extra bits).
struct InfV4 {
    uint32_t x, y, z, w;
};
struct InfBits {
    const InfV4 *v;
    uint32_t nv, vi, wi;  // vectors holding data, index of `cur`, next word of `cur`
    InfV4 cur, n1, n2;    // the vector being consumed, the next two
    uint32_t skip, n;     // data start in vector 0 (bytes), data length (bytes)
    uint64_t bb;          // bit buffer (LSB = next bit)
    int nb;               // valid bits in bb

    SVT_HD InfV4 ld(uint32_t i) const { return i < nv ? v[i] : InfV4{0u, 0u, 0u, 0u}; }
    SVT_HD void init(const InfV4 *vecs, uint32_t skip_bytes, uint32_t len) {
        v = vecs;
        skip = skip_bytes;
        n = len;
        nv = (skip_bytes + len + 15u) >> 4;
        cur = ld(0);
        n1 = ld(1);
        n2 = ld(2);
        vi = 0;
        wi = skip_bytes >> 2;
        bb = 0;
        nb = 0;
        fill();
        drop(8 * (int)(skip_bytes & 3u));
    }
    SVT_HD void fill() {
        while (nb <= 32) {
            const uint32_t x = wi == 0 ? cur.x : wi == 1 ? cur.y : wi == 2 ? cur.z : cur.w;
            bb |= (uint64_t)x << nb;
            nb += 32;
            if (++wi == 4) {
                cur = n1;
                n1 = n2;
                vi++;
                n2 = ld(vi + 2);
                wi = 0;
            }
        }
    }
    SVT_HD bool past() const {   // consumed more than n bytes
        return 32ull * (4ull * vi + wi) - (uint64_t)nb - 8ull * skip > 8ull * n;
    }
    SVT_HD uint32_t peek(int k) { return (uint32_t)(bb & ((1ull << k) - 1)); }
    SVT_HD void drop(int k) { bb >>= k; nb -= k; }
    SVT_HD uint32_t get(int k) {   // k <= 32, after fill() guaranteeing k bits
        const uint32_t v_ = peek(k);
        drop(k);
        return v_;
    }
};

SVT_HD uint32_t inf_rev(uint32_t code, int len) {   // reverse the low len bits
    uint32_t r = 0;
    for (int i = 0; i < len; i++) r |= ((code >> i) & 1u) << (len - 1 - i);
    return r;
}

// Build a table from n code lengths: primary entries (tab, 1 << bits) + slow-path arrays.
// False for a code zlib's inflate_table rejects (inftrees.c): over-subscribed, or incomplete
// where it is not allowed -- kind INF_CODES (the code-length code) never, INF_LENS (litlen and
// distance codes) only for a single code of length 1; a code with no symbols at all is built
// (every lookup fails, as zlib's "invalid code" table does).  INF_FIXED: the fixed codes (their
// 30 distance codes of 5 bits are short of the 32 zlib builds; the 2 unused ones never occur).
constexpr int INF_FIXED = 0, INF_CODES = 1, INF_LENS = 2;
SVT_HD bool inf_build(const uint8_t *len, int n, const InfTab tab, int bits, uint16_t *cnt, uint16_t *sym,
                      uint16_t *offs, int kind) {
    for (int i = 0; i < 16; i++) cnt[i] = 0;
    for (int s = 0; s < n; s++) cnt[len[s]]++;
    cnt[0] = 0;
    int left = 1, max = 0;
    for (int l = 1; l < 16; l++) {
        left <<= 1;
        left -= cnt[l];
        if (left < 0) return false;   // over-subscribed
        if (cnt[l]) max = l;
    }
    if (kind != INF_FIXED && max > 0 && left > 0 && (kind == INF_CODES || max != 1)) return false;   // incomplete
    offs[1] = 0;
    for (int l = 1; l < 15; l++) offs[l + 1] = (uint16_t)(offs[l] + cnt[l]);
    for (int s = 0; s < n; s++)
        if (len[s]) sym[offs[len[s]]++] = (uint16_t)s;
    // primary table: canonical codes in (length, symbol) order
    for (int i = 0; i < (1 << bits); i++) tab[i] = 0;
    uint32_t code = 0;
    int k = 0;
    for (int l = 1; l < 16; l++) {
        for (int c = 0; c < cnt[l]; c++, k++, code++) {
            if (l > bits) continue;
            const uint32_t r = inf_rev(code, l);
            const uint16_t e = (uint16_t)(sym[k] | (l << 9));
            for (uint32_t i = r; i < (1u << bits); i += 1u << l) tab[i] = e;
        }
        code <<= 1;
    }
    return true;
}

// Decode one symbol (after fill()): primary table, else the canonical walk over lengths > bits.
SVT_HD int inf_decode(InfBits &br, const InfTab tab, int bits, const uint16_t *cnt, const uint16_t *sym) {
    const uint16_t e = tab[br.peek(bits)];
    if (e) {
        br.drop(e >> 9);
        return e & 0x1ff;
    }
    int code = 0, first = 0, index = 0;
    for (int l = 1; l < 16; l++) {
        code |= (int)((br.bb >> (l - 1)) & 1u);
        const int c = cnt[l];
        if (code - c < first) {
            br.drop(l);
            return sym[index + (code - first)];
        }
        index += c;
        first += c;
        first <<= 1;
        code <<= 1;
    }
    return -1;   // no code of this stream matches (incomplete code)
}

// RFC 1951 3.2.5 length / distance bases and extra bits
// (arithmetic forms of the RFC's tables: 3, 4, .. 10, 11, 13, .. 227, 258 and 1, 2, 3, 4, 5, 7, .. 24577)
SVT_HD int inf_lext(int i) { return i < 8 || i == 28 ? 0 : (i - 4) >> 2; }
SVT_HD uint32_t inf_lbase(int i) {
    return i < 8 ? 3u + (uint32_t)i : i == 28 ? 258u : ((4u + (uint32_t)(i & 3)) << inf_lext(i)) + 3u;
}
SVT_HD int inf_dext(int i) { return i < 4 ? 0 : (i - 2) >> 1; }
SVT_HD uint32_t inf_dbase(int i) { return i < 4 ? 1u + (uint32_t)i : ((2u + (uint32_t)(i & 1)) << inf_dext(i)) + 1u; }
// the code-length code's transmission order, 16 17 18 0 8 7 9 6 10 5 11 4 12 3 13 2 14 1 15, 5 bits each
SVT_HD int inf_ord(int i) {
    const uint64_t lo = 16ull | 17ull << 5 | 18ull << 10 | 0ull << 15 | 8ull << 20 | 7ull << 25 | 9ull << 30 | 6ull << 35 |
                        10ull << 40 | 5ull << 45 | 11ull << 50 | 4ull << 55;
    const uint64_t hi = 12ull | 3ull << 5 | 13ull << 10 | 2ull << 15 | 14ull << 20 | 1ull << 25 | 15ull << 30;
    return (int)((i < 12 ? lo >> (5 * i) : hi >> (5 * (i - 12))) & 31u);
}

// Inflate one raw DEFLATE stream of clen bytes, starting `skip` (< 16) bytes into the 16-B
// aligned `in`, to out[0..ulen).  Returns INF_OK only when the stream ends (BFINAL block done)
// with exactly ulen bytes written and no read past clen.
SVT_HD int inf_block(const InfV4 *in, uint32_t skip, uint32_t clen, uint8_t *out, uint32_t ulen, const InfFast &F,
                     InfSlow &S) {
    InfBits br;
    br.init(in, skip, clen);
    uint32_t op = 0;
    for (;;) {
        br.fill();
        const uint32_t hdr = br.get(3);
        const uint32_t type = hdr >> 1;
        if (type == 0) {   // stored
            br.drop(br.nb & 7);   // to the byte boundary
            br.fill();
            const uint32_t L = br.get(16), NL = br.get(16);
            if ((L ^ 0xffffu) != NL) return INF_EDATA;
            if (op + L > ulen) return INF_EOUT;
            for (uint32_t i = 0; i < L; i++) {
                br.fill();
                out[op++] = (uint8_t)br.get(8);
            }
        } else if (type == 1 || type == 2) {
            if (type == 1) {   // fixed codes (RFC 1951 3.2.6)
                for (int s = 0; s < 288; s++) S.len[s] = (uint8_t)(s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8);
                for (int s = 0; s < 30; s++) S.len[288 + s] = 5;
                inf_build(S.len, 288, F.lit, IF_LB, S.lcnt, S.lsym, S.offs, INF_FIXED);
                inf_build(S.len + 288, 30, F.dst, IF_DB, S.dcnt, S.dsym, S.offs, INF_FIXED);
            } else {           // dynamic codes (3.2.7)
                br.fill();
                const int nlen = (int)br.get(5) + 257, ndist = (int)br.get(5) + 1, ncode = (int)br.get(4) + 4;
                if (nlen > 286 || ndist > 30) return INF_EDATA;
                for (int i = 0; i < 19; i++) S.cl[i] = 0;
                for (int i = 0; i < ncode; i++) {
                    br.fill();
                    S.cl[inf_ord(i)] = (uint8_t)br.get(3);
                }
                // the code-length code: 7-bit table in the litlen table's place
                if (!inf_build(S.cl, 19, F.lit, 7, S.lcnt, S.lsym, S.offs, INF_CODES)) return INF_EDATA;
                int i = 0;
                while (i < nlen + ndist) {
                    br.fill();
                    const int s = inf_decode(br, F.lit, 7, S.lcnt, S.lsym);
                    if (s < 0) return INF_EDATA;
                    if (s < 16) {
                        S.len[i++] = (uint8_t)s;
                        continue;
                    }
                    uint8_t v = 0;
                    int rep;
                    if (s == 16) {
                        if (i == 0) return INF_EDATA;
                        v = S.len[i - 1];
                        rep = 3 + (int)br.get(2);
                    } else if (s == 17) {
                        rep = 3 + (int)br.get(3);
                    } else {
                        rep = 11 + (int)br.get(7);
                    }
                    if (i + rep > nlen + ndist) return INF_EDATA;
                    while (rep--) S.len[i++] = v;
                }
                if (S.len[256] == 0) return INF_EDATA;   // no end-of-block code
                // (the dist lengths move to 288.. so that both live in S.len while building)
                for (int k = ndist - 1; k >= 0; k--) S.len[288 + k] = S.len[nlen + k];
                for (int k = nlen; k < 288; k++) S.len[k] = 0;
                if (!inf_build(S.len, 288, F.lit, IF_LB, S.lcnt, S.lsym, S.offs, INF_LENS)) return INF_EDATA;
                if (!inf_build(S.len + 288, ndist, F.dst, IF_DB, S.dcnt, S.dsym, S.offs, INF_LENS)) return INF_EDATA;
            }
            // literals are combined into 4-byte stores at 4-byte aligned output addresses (wc holds
            // the wn bytes of the current word, from out[op - wn]); a match or the block's end
            // flushes them first (the copy reads them back)
            uint32_t wc = 0, wn = 0;
            auto flush = [&]() {
                for (uint32_t i = 0; i < wn; i++) out[op - wn + i] = (uint8_t)(wc >> (8 * i));
                wc = 0;
                wn = 0;
            };
            for (;;) {   // literals / lengths until end of block
                br.fill();
                const int s = inf_decode(br, F.lit, IF_LB, S.lcnt, S.lsym);
                if (s < 256) {
                    if (s < 0) return INF_EDATA;
                    if (op >= ulen) return INF_EOUT;
                    if (wn == 0 && (((uintptr_t)(out + op)) & 3u) != 0u) {
                        out[op++] = (uint8_t)s;   // (not yet at a word boundary)
                        continue;
                    }
                    wc |= (uint32_t)s << (8 * wn);
                    op++;
                    if (++wn == 4) {
                        *reinterpret_cast<uint32_t *>(out + op - 4) = wc;
                        wc = 0;
                        wn = 0;
                    }
                    continue;
                }
                flush();
                if (s == 256) break;
                const int li = s - 257;
                if (li >= 29) return INF_EDATA;
                const uint32_t len = inf_lbase(li) + br.get(inf_lext(li));
                br.fill();
                const int d = inf_decode(br, F.dst, IF_DB, S.dcnt, S.dsym);
                if (d < 0 || d >= 30) return INF_EDATA;
                const uint32_t dist = inf_dbase(d) + br.get(inf_dext(d));
                if (dist > op) return INF_EDATA;
                if (op + len > ulen) return INF_EOUT;
                uint32_t k = 0;
                if (dist >= 8)   // 8 bytes a step: the loads of a step issued before its stores
                    for (; k + 8 <= len; k += 8, op += 8) {
                        uint8_t t[8];
#pragma unroll
                        for (int i = 0; i < 8; i++) t[i] = out[op - dist + i];
#pragma unroll
                        for (int i = 0; i < 8; i++) out[op + i] = t[i];
                    }
                for (; k < len; k++, op++) out[op] = out[op - dist];
            }
        } else {
            return INF_EDATA;
        }
        if (br.past()) return INF_EIN;
        if (hdr & 1u) break;   // BFINAL
    }
    return op == ulen ? INF_OK : INF_EOUT;
}
