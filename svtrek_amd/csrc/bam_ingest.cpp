// bam_ingest.cpp -- BGZF/BAM reader -> columnar pileup (svtrek_host.h).
//
// What the reference gets from htslib on this path (refinement.c:114-120) is, per
// yielded record: core.tid, core.pos, core.flag (via bam_endpos, used by the region
// overlap test), n_cigar and the CIGAR -- after bam_read1 has restored a >65535-op
// CIGAR from its CG:B,I tag (htslib bam_tag2cigar) -- plus the two words the soft-clip
// tests read (cigar[n_cigar-1] and cigar[0], which for n_cigar == 0 land in the padded
// read name / the SEQ bytes of htslib's bam1_t data layout).  This reader extracts
// exactly those, once per file: BGZF blocks are inflated in parallel in bounded chunks,
// records are parsed sequentially, and SEQ/QUAL/aux are dropped.
#include <zlib.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "svtrek_host.h"

namespace {

constexpr uint32_t OP_M = 0, OP_D = 2, OP_N = 3, OP_S = 4, OP_EQ = 7, OP_X = 8;

inline uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
inline uint16_t rd16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }

struct BgzfReader {
    FILE *f = nullptr;
    int threads = 1;
    std::vector<uint8_t> comp;     // compressed bytes not yet consumed
    bool eof = false;
    std::string err;

    // Append the next batch of inflated blocks to `out`; false at end of file / on error.
    bool next(std::vector<uint8_t> &out) {
        const size_t CHUNK = 64u << 20;
        if (!eof) {
            size_t old = comp.size();
            comp.resize(old + CHUNK);
            size_t got = fread(comp.data() + old, 1, CHUNK, f);
            comp.resize(old + got);
            if (got < CHUNK) eof = true;
        }
        // index complete blocks
        struct Blk { size_t off, clen, ulen, cdata; };
        std::vector<Blk> blks;
        size_t p = 0;
        while (p + 18 <= comp.size()) {
            const uint8_t *h = comp.data() + p;
            if (h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) { err = "not a BGZF file (bad gzip header)"; return false; }
            uint16_t xlen = rd16(h + 10);
            if (p + 12 + xlen > comp.size()) break;
            size_t bsize = 0;
            for (size_t x = 0; x + 4 <= xlen;) {
                const uint8_t *sf = h + 12 + x;
                uint16_t slen = rd16(sf + 2);
                if (sf[0] == 66 && sf[1] == 67 && slen == 2) bsize = (size_t)rd16(sf + 4) + 1;
                x += 4 + slen;
            }
            if (!bsize) { err = "BGZF block without BC subfield"; return false; }
            if (p + bsize > comp.size()) break;
            size_t cdata = p + 12 + xlen, clen = bsize - xlen - 20;
            uint32_t isize = rd32(comp.data() + p + bsize - 4);
            blks.push_back({p, clen, isize, cdata});
            p += bsize;
        }
        if (blks.empty()) {
            if (eof && !comp.empty()) { err = "truncated BGZF block at end of file"; return false; }
            return !(eof && comp.empty()) && !comp.empty() ? false : false;
        }
        std::vector<size_t> uoff(blks.size() + 1, 0);
        for (size_t i = 0; i < blks.size(); i++) uoff[i + 1] = uoff[i] + blks[i].ulen;
        size_t base = out.size();
        out.resize(base + uoff.back());
        std::vector<int> bad(blks.size(), 0);
        auto work = [&](int t) {
            z_stream zs;
            memset(&zs, 0, sizeof zs);
            if (inflateInit2(&zs, -15) != Z_OK) { bad[0] = 1; return; }
            for (size_t i = (size_t)t; i < blks.size(); i += (size_t)threads) {
                inflateReset(&zs);
                zs.next_in = comp.data() + blks[i].cdata;
                zs.avail_in = (uInt)blks[i].clen;
                zs.next_out = out.data() + base + uoff[i];
                zs.avail_out = (uInt)blks[i].ulen;
                int rc = inflate(&zs, Z_FINISH);
                if (rc != Z_STREAM_END || zs.total_out != blks[i].ulen) bad[i] = 1;
                zs.total_out = 0;
            }
            inflateEnd(&zs);
        };
        int nt = std::max(1, std::min<int>(threads, (int)blks.size()));
        if (nt == 1) work(0);
        else {
            std::vector<std::thread> th;
            for (int t = 0; t < nt; t++) th.emplace_back(work, t);
            for (auto &x : th) x.join();
        }
        for (size_t i = 0; i < blks.size(); i++)
            if (bad[i]) { err = "corrupt BGZF block (inflate failed)"; return false; }
        comp.erase(comp.begin(), comp.begin() + (ptrdiff_t)p);
        return true;
    }
};

}  // namespace

struct svth_bam {
    std::vector<std::string> names;
    std::vector<int64_t> tid_off;
    std::vector<int32_t> pos, endpos;
    std::vector<uint64_t> cig_off;
    std::vector<uint32_t> cigar;
    std::vector<uint8_t> clip;
    int64_t n_records = 0, n_cg = 0;
};

namespace {

struct RawRead { int32_t tid, pos, endpos; uint64_t off; uint32_t n; uint8_t clip; int64_t seq; };

// htslib bam_tag2cigar's conditions: n_cigar > 0, tid >= 0, pos >= 0, cigar[0] == <l_seq>S,
// a CG tag of type B,I (or B,i) with at least n_cigar elements and fewer than 2^29.
bool find_cg(const uint8_t *aux, const uint8_t *end, const uint8_t **arr, uint32_t *cnt) {
    const uint8_t *p = aux;
    while (p + 3 <= end) {
        char t0 = (char)p[0], t1 = (char)p[1], ty = (char)p[2];
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
            char sub = (char)p[0];
            uint32_t n = rd32(p + 1);
            size_t es = (sub == 'c' || sub == 'C') ? 1 : (sub == 's' || sub == 'S') ? 2
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

}  // namespace

extern "C" {

svth_bam *svth_bam_read(const char *path, int threads, char *err, size_t errcap) {
    auto fail = [&](const std::string &m) -> svth_bam * {
        if (err && errcap) snprintf(err, errcap, "%s", m.c_str());
        return nullptr;
    };
    FILE *f = fopen(path, "rb");
    if (!f) return fail(std::string("cannot open BAM: ") + path);
    BgzfReader rd;
    rd.f = f;
    rd.threads = threads < 1 ? 1 : threads;
    std::vector<uint8_t> buf;
    size_t at = 0;
    auto need = [&](size_t k) -> bool {
        while (buf.size() - at < k) {
            if (at > (16u << 20)) { buf.erase(buf.begin(), buf.begin() + (ptrdiff_t)at); at = 0; }
            if (!rd.next(buf)) return false;
        }
        return true;
    };
    svth_bam *b = new svth_bam();
    // header
    if (!need(8) || memcmp(buf.data() + at, "BAM\1", 4) != 0) {
        fclose(f); delete b;
        return fail(rd.err.empty() ? "not a BAM file" : rd.err);
    }
    uint32_t l_text = rd32(buf.data() + at + 4);
    at += 8;
    if (!need((size_t)l_text + 4)) { fclose(f); delete b; return fail("truncated BAM header"); }
    at += l_text;
    int32_t n_ref = (int32_t)rd32(buf.data() + at);
    at += 4;
    if (n_ref < 0) { fclose(f); delete b; return fail("bad n_ref"); }
    for (int32_t i = 0; i < n_ref; i++) {
        if (!need(4)) { fclose(f); delete b; return fail("truncated reference list"); }
        uint32_t ln = rd32(buf.data() + at);
        if (!need(4 + (size_t)ln + 4)) { fclose(f); delete b; return fail("truncated reference list"); }
        b->names.emplace_back((const char *)buf.data() + at + 4, ln ? ln - 1 : 0);
        at += 4 + ln + 4;
    }
    std::vector<RawRead> rr;
    std::vector<uint32_t> arena;
    int64_t seq = 0;
    for (;;) {
        if (buf.size() - at < 4 && !need(4)) break;   // clean EOF
        uint32_t bs = rd32(buf.data() + at);
        if (bs < 32) { fclose(f); delete b; return fail("corrupt BAM record (block_size < 32)"); }
        if (!need(4 + (size_t)bs)) { fclose(f); delete b; return fail(rd.err.empty() ? "truncated BAM record" : rd.err); }
        const uint8_t *r = buf.data() + at + 4, *rend = r + bs;
        at += 4 + bs;
        b->n_records++;
        int32_t tid = (int32_t)rd32(r), pos = (int32_t)rd32(r + 4);
        uint32_t l_qname = r[8];
        uint16_t n_cig = rd16(r + 12), flag = rd16(r + 14);
        int32_t l_seq = (int32_t)rd32(r + 16);
        if (tid < 0 || tid >= n_ref) continue;      // never yielded by a tid >= 0 region query
        const uint8_t *qn = r + 32, *cg = qn + l_qname;
        if (cg + 4ull * n_cig > rend || l_seq < 0) { fclose(f); delete b; return fail("corrupt BAM record"); }
        const uint8_t *after = cg + 4ull * n_cig;    // SEQ starts here
        const uint8_t *aux = after + (size_t)(l_seq + 1) / 2 + (size_t)l_seq;
        const uint8_t *src = cg;
        uint32_t n = n_cig;
        if (n_cig > 0 && pos >= 0 && (rd32(cg) & 0xfu) == OP_S && (int64_t)(rd32(cg) >> 4) == l_seq && aux <= rend) {
            const uint8_t *arr;
            uint32_t cnt;
            if (find_cg(aux, rend, &arr, &cnt) && cnt >= n_cig && cnt < (1u << 29)) {
                src = arr; n = cnt; b->n_cg++;
            }
        }
        RawRead x;
        x.tid = tid; x.pos = pos; x.off = arena.size(); x.n = n; x.seq = seq++;
        arena.resize(arena.size() + n);
        if (n) memcpy(arena.data() + x.off, src, 4ull * n);
        int64_t rl = 0;
        if (!(flag & 4))
            for (uint32_t i = 0; i < n; i++) {
                uint32_t op = arena[x.off + i] & 0xfu;
                if (op == OP_M || op == OP_D || op == OP_N || op == OP_EQ || op == OP_X) rl += arena[x.off + i] >> 4;
            }
        x.endpos = (int32_t)(pos + (rl ? rl : 1));
        // Soft-clip test words as the reference reads them through bam1_t.data: the qname is
        // padded with NULs to a multiple of 4 (htslib l_extranul), so cigar[-1] is the last
        // 4 bytes of the padded name and cigar[0] of an empty CIGAR is the first SEQ byte.
        uint8_t c = 0;
        if (n) {
            if ((arena[x.off + n - 1] & 0xfu) == OP_S) c |= SVT_CLIP_LAST_S;
            if ((arena[x.off] & 0xfu) == OP_S) c |= SVT_CLIP_FIRST_S;
        } else {
            uint32_t padded = (l_qname + 3u) & ~3u;
            uint8_t lastw0 = padded >= 4 ? (padded - 4 < l_qname ? qn[padded - 4] : 0) : 0;
            if ((lastw0 & 0xfu) == OP_S) c |= SVT_CLIP_LAST_S;
            if (after < rend && (after[0] & 0xfu) == OP_S) c |= SVT_CLIP_FIRST_S;
        }
        x.clip = c;
        if (pos < 0) continue;
        rr.push_back(x);
    }
    fclose(f);
    if (!rd.err.empty()) { delete b; return fail(rd.err); }
    // columnar, per tid sorted by pos (file order among equal pos; order is irrelevant)
    std::vector<size_t> idx(rr.size());
    std::iota(idx.begin(), idx.end(), 0);
    std::stable_sort(idx.begin(), idx.end(), [&](size_t a, size_t c) {
        return rr[a].tid != rr[c].tid ? rr[a].tid < rr[c].tid : rr[a].pos < rr[c].pos;
    });
    b->tid_off.assign((size_t)n_ref + 1, 0);
    b->pos.resize(rr.size()); b->endpos.resize(rr.size()); b->clip.resize(rr.size());
    b->cig_off.resize(rr.size() + 1);
    b->cigar.resize(arena.size());
    uint64_t w = 0;
    for (size_t k = 0; k < idx.size(); k++) {
        const RawRead &x = rr[idx[k]];
        b->tid_off[(size_t)x.tid + 1]++;
        b->pos[k] = x.pos; b->endpos[k] = x.endpos; b->clip[k] = x.clip;
        b->cig_off[k] = w;
        if (x.n) memcpy(b->cigar.data() + w, arena.data() + x.off, 4ull * x.n);
        w += x.n;
    }
    b->cig_off[rr.size()] = w;
    for (int32_t t = 0; t < n_ref; t++) b->tid_off[(size_t)t + 1] += b->tid_off[(size_t)t];
    return b;
}

void svth_bam_free(svth_bam *b) { delete b; }

void svth_bam_view(const svth_bam *b, svt_pileup_view *v) {
    v->n_targets = (int32_t)b->names.size();
    v->tid_off = b->tid_off.data();
    v->pos = b->pos.data();
    v->endpos = b->endpos.data();
    v->cig_off = b->cig_off.data();
    v->cigar = b->cigar.data();
    v->clip = b->clip.data();
}

int32_t svth_bam_n_targets(const svth_bam *b) { return (int32_t)b->names.size(); }
const char *svth_bam_target_name(const svth_bam *b, int32_t t) {
    return (t >= 0 && (size_t)t < b->names.size()) ? b->names[(size_t)t].c_str() : nullptr;
}
int64_t svth_bam_n_records(const svth_bam *b) { return b->n_records; }
int64_t svth_bam_n_cg_restored(const svth_bam *b) { return b->n_cg; }

}  // extern "C"
