// bam_ingest.cpp -- BGZF/BAM reader -> columnar pileup (svtrek_host.h).
//
// What the reference gets from htslib on this path (refinement.c:114-120) is, per
// yielded record: core.tid, core.pos, core.flag (via bam_endpos, used by the region
// overlap test), n_cigar and the CIGAR -- after bam_read1 has restored a >65535-op
// CIGAR from its CG:B,I tag (htslib bam_tag2cigar) -- plus the two words the soft-clip
// tests read (cigar[n_cigar-1] and cigar[0], which for n_cigar == 0 land in the padded
// read name / the SEQ bytes of htslib's bam1_t data layout).  This reader extracts
// exactly those, once per file, in bounded chunks:
//   1. parallel raw-inflate of the chunk's BGZF blocks (libdeflate if present, else zlib;
//      T threads);
//   2. a sequential scan of the record boundaries (4 bytes per record);
//   3. parallel per-record extraction in two passes (CIGAR lengths incl. CG tags, then
//      copies into the final arrays at prefix-summed offsets).
// A coordinate-sorted BAM (the only kind that has a BAI) needs no reordering; other
// files are stably sorted by (tid, pos) at the end.  SEQ/QUAL/aux are never copied.
#include <dlfcn.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <future>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "svtrek_host.h"
#include "svt_bamrec.h"

namespace {



inline uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
inline uint16_t rd16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }

template <typename F>
void parallel_for(int threads, size_t n, F &&f) {   // f(begin, end) over contiguous slices
    const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)std::max(threads, 1), n / 4096 + 1));
    if (T == 1) { f((size_t)0, n); return; }
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++) th.emplace_back([&, t] { f(n * t / T, n * (t + 1) / T); });
    for (auto &x : th) x.join();
}

// Raw-DEFLATE block decoder: libdeflate when the system has it (libdeflate.so.0, bound at
// run time through its stable C API: alloc / deflate_decompress / free), zlib otherwise.
struct Inflater {
    using alloc_t = void *(*)();
    using dec_t = int (*)(void *, const void *, size_t, void *, size_t, size_t *);
    using free_t = void (*)(void *);
    alloc_t ld_alloc = nullptr;
    dec_t ld_dec = nullptr;
    free_t ld_free = nullptr;
    Inflater() {
        if (getenv("SVTREK_NO_LIBDEFLATE")) return;
        void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        ld_alloc = (alloc_t)dlsym(h, "libdeflate_alloc_decompressor");
        ld_dec = (dec_t)dlsym(h, "libdeflate_deflate_decompress");
        ld_free = (free_t)dlsym(h, "libdeflate_free_decompressor");
        if (!ld_alloc || !ld_dec || !ld_free) ld_alloc = nullptr;
    }
    bool fast() const { return ld_alloc != nullptr; }
};
const Inflater &inflater() {
    static const Inflater inf;
    return inf;
}

// Growable byte buffer without value-initialisation; view() points it at a buffer owned by the
// reader (the device-inflated batches are handed over without a copy).
struct Bytes {
    uint8_t *p = nullptr;
    size_t n = 0, cap = 0;
    Bytes() = default;
    Bytes(const Bytes &) = delete;
    Bytes &operator=(const Bytes &) = delete;
    ~Bytes() {
        if (owned) free(p);
    }
    size_t size() const { return n; }
    uint8_t *data() { return p; }
    const uint8_t *data() const { return p; }
    bool resize(size_t m) {
        if (m > cap) {
            const size_t c = std::max(m, cap + cap / 2);
            uint8_t *q = (uint8_t *)(owned ? realloc(p, c) : malloc(c));
            if (!q) return false;
            if (!owned && n) memcpy(q, p, n);
            p = q;
            cap = c;
            owned = true;
        }
        n = m;
        return true;
    }
    void erase_front(size_t k) {
        if (k) memmove(p, p + k, n - k);
        n -= k;
    }
    void clear() { n = 0; }
    bool owned = true;   // false: a view of a buffer someone else frees (view())
    void view(uint8_t *q, size_t m) {
        if (owned) free(p);
        p = q;
        n = cap = m;
        owned = false;
    }
};

struct BgzfReader {
    FILE *f = nullptr;
    int threads = 1;
    std::vector<uint8_t> comp;     // compressed bytes not yet consumed
    bool eof = false;
    std::string err;
    // device inflate (svth_inflater): batches of ~`batch` compressed bytes, read with parallel
    // preads into a reused input buffer and inflated by inf->inflate into one of two reused
    // output buffers (from inf->alloc: pinned host memory, so the copies to and from the device
    // run at full speed); the next batch is read and inflated by a helper thread while the
    // caller parses the current one
    const svth_inflater *inf = nullptr;
    static constexpr size_t HEAD = 64ull << 20;   // room in front of a batch for the previous one's tail
    struct Buf {
        uint8_t *p = nullptr;
        size_t cap = 0;
        bool pinned = false;   // from inf->alloc (else malloc: pinned memory was refused)
    };
    Buf cins[2], outs[2];  // compressed input (one inflated, one being read); output (one parsed, one filled)
    size_t cin_n[2] = {0, 0};
    int read_i = 0, fill_i = 0;   // the input / output buffer the next batch goes to
    // the partial block at the end of the last batch read: cins[carry_i][carry_p, +carry_n)
    int carry_i = 0;
    size_t carry_p = 0, carry_n = 0;
    struct Comp {                 // a batch read and scanned: its blocks in cins[i][0, p)
        int i = 0;
        size_t p = 0, u = 0;
        std::vector<svt_bgzf_block> blks;
        bool ok = false;
        std::string err;
    };
    std::future<Comp> pending_comp;
    uint64_t foff = 0, fsize = 0;
    struct Batch {
        uint8_t *p = nullptr;   // outs[i].p: HEAD bytes, then n inflated bytes
        size_t n = 0;
        bool ok = false;
        std::string err;
    };
    std::future<Batch> pending;
    // stage times (s): read, header scan, buffer allocation (reader, inflater), inflate, parser
    // waiting on a batch
    double t_read = 0, t_scan = 0, t_alloc_r = 0, t_alloc = 0, t_inflate = 0, t_wait = 0;
    static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

    ~BgzfReader() {
        drop_pending();
        for (Buf *b : {&cins[0], &cins[1], &outs[0], &outs[1]}) release(*b);
    }
    void drop_pending() {
        if (pending.valid()) (void)pending.get();
        if (pending_comp.valid()) (void)pending_comp.get();
    }
    void release(Buf &b) {
        if (b.p) {
            if (b.pinned) inf->release(inf->user, b.p);
            else free(b.p);
        }
        b = Buf{};
    }
    // grow to >= need, keeping the first `keep` bytes; pinned memory when the inflater offers it,
    // pageable memory when pinning is refused (the copies are only slower)
    bool reserve(Buf &b, size_t need, size_t keep) {
        if (need <= b.cap) return true;
        const size_t c = std::max(need, b.cap + b.cap / 2);
        bool pinned = inf && inf->alloc && inf->release;
        uint8_t *q = pinned ? (uint8_t *)inf->alloc(inf->user, c) : nullptr;
        if (!q) {
            pinned = false;
            q = (uint8_t *)malloc(c);
        }
        if (!q) return false;
        if (keep) memcpy(q, b.p, keep);
        release(b);
        b.p = q;
        b.cap = c;
        b.pinned = pinned;
        return true;
    }

    // Continue at compressed file offset `coff` (a BGZF block start).
    bool seek(uint64_t coff) {
        drop_pending();
        comp.clear();
        cin_n[0] = cin_n[1] = 0;
        carry_n = 0;
        foff = coff;
        eof = false;
        if (fseeko(f, (off_t)coff, SEEK_SET) != 0) { err = "cannot seek in BAM (BAI offset past the end?)"; return false; }
        return true;
    }

    // Append the next ~want compressed bytes to buffer b (holding n), `threads` preads at once.
    bool read_batch(Buf &b, size_t &n, size_t want) {
        if (foff >= fsize) { eof = true; return true; }
        want = (size_t)std::min<uint64_t>(want, fsize - foff);
        const double t0 = now();
        if (!reserve(b, n + want + 64, n)) { err = "out of host memory"; return false; }
        const double t1 = now();
        t_alloc_r += t1 - t0;
        const int fd = fileno(f);
        std::atomic<int> bad{0};
        uint8_t *dst = b.p + n;
        const uint64_t at = foff;
        parallel_for(threads, want, [&](size_t a, size_t e) {
            for (size_t o = a; o < e;) {
                const ssize_t r = pread(fd, dst + o, e - o, (off_t)(at + o));
                if (r <= 0) { bad = 1; return; }
                o += (size_t)r;
            }
        });
        t_read += now() - t1;
        if (bad) { err = "cannot read BAM"; return false; }
        n += want;
        foff += want;
        if (foff >= fsize) eof = true;
        return true;
    }

    // Read and scan the next batch into cins[read_i] (the previous batch's partial block first).
    Comp read_next() {
        Comp c;
        c.i = read_i;
        Buf &b = cins[read_i];
        size_t &n = cin_n[read_i];
        const size_t want = inf->batch_bytes ? inf->batch_bytes : (1ull << 30);
        n = 0;
        if (carry_n) {
            const double t0 = now();
            if (!reserve(b, carry_n + want + 64, 0)) { c.err = "out of host memory"; return c; }
            t_alloc_r += now() - t0;
            memcpy(b.p, cins[carry_i].p + carry_p, carry_n);
            n = carry_n;
        }
        size_t p = 0, u = 0;
        for (;;) {
            if (!eof && !read_batch(b, n, want)) { c.err = err; return c; }
            const double ts = now();
            while (p + 18 <= n) {
                const uint8_t *h = b.p + p;
                if (h[0] != 31 || h[1] != 139 || h[2] != 8 || !(h[3] & 4)) { c.err = "not a BGZF file (bad gzip header)"; return c; }
                const uint16_t xlen = rd16(h + 10);
                if (p + 12 + xlen > n) break;
                size_t bsize = 0;
                for (size_t x = 0; x + 4 <= xlen;) {
                    const uint8_t *sf = h + 12 + x;
                    const uint16_t slen = rd16(sf + 2);
                    if (sf[0] == 66 && sf[1] == 67 && slen == 2) bsize = (size_t)rd16(sf + 4) + 1;
                    x += 4 + slen;
                }
                if (!bsize || bsize < (size_t)xlen + 20) { c.err = "BGZF block without BC subfield"; return c; }
                if (p + bsize > n) break;
                svt_bgzf_block k;
                k.coff = p + 12 + xlen;
                k.clen = (uint32_t)(bsize - xlen - 20);
                k.uoff = u;
                k.ulen = rd32(b.p + p + bsize - 4);
                c.blks.push_back(k);
                u += k.ulen;
                p += bsize;
            }
            t_scan += now() - ts;
            if (!c.blks.empty() || eof) break;   // (else a single block larger than what was read so far)
        }
        if (c.blks.empty() && n) { c.err = "truncated BGZF block at end of file"; return c; }
        c.p = p;
        c.u = u;
        c.ok = true;
        carry_i = read_i;
        carry_p = p;
        carry_n = n - p;
        read_i ^= 1;
        return c;
    }

    // Inflate the next batch (helper thread), the batch after it being read meanwhile; ok && n ==
    // 0 at end of file.
    Batch produce() {
        Batch b;
        Comp c = pending_comp.valid() ? pending_comp.get() : read_next();
        // a batch of empty blocks only (ISIZE 0 each) is skipped, not taken for the end of file
        while (c.ok && !c.blks.empty() && c.u == 0) {
            if (eof && !carry_n) { c.blks.clear(); break; }
            c = read_next();
        }
        if (!c.ok) { b.err = c.err; return b; }
        if (c.blks.empty()) { b.ok = true; return b; }   // end of file
        if (!eof || carry_n) pending_comp = std::async(std::launch::async, [this] { return read_next(); });
        Buf &o = outs[fill_i];
        double t0 = now();
        if (!reserve(o, HEAD + c.u + 16, 0)) { b.err = "out of host memory"; return b; }
        double t1 = now();
        t_alloc += t1 - t0;
        char e[256] = {0};
        const int rc = inf->inflate(inf->user, cins[c.i].p, c.p, c.blks.data(), c.blks.size(), o.p + HEAD, c.u, e, sizeof e);
        t_inflate += now() - t1;
        if (rc != 0) {
            b.err = e[0] ? e : "BGZF inflate failed";
            return b;
        }
        b.p = o.p;
        b.n = c.u;
        b.ok = true;
        fill_i ^= 1;
        return b;
    }

    // Device path of next(): the pending batch (or a synchronous first one) becomes the buffer,
    // the unconsumed tail [at, size) moved in front of it; the batch after it starts, into the
    // output buffer the parser just left.
    bool next_device(Bytes &out, size_t &at) {
        const double tw = now();
        Batch b = pending.valid() ? pending.get() : produce();
        t_wait += now() - tw;
        if (!b.ok) { err = b.err; return false; }
        if (b.n == 0) return false;   // end of file
        const size_t tail = out.size() - at;
        if (tail > HEAD) { err = "a BAM record longer than 64 MiB"; return false; }
        memcpy(b.p + HEAD - tail, out.data() + at, tail);
        out.view(b.p, HEAD + b.n);   // (the reader owns the buffer)
        at = HEAD - tail;
        pending = std::async(std::launch::async, [this] { return produce(); });
        return true;
    }

    // Make more inflated bytes available in out (consumed up to `at`); false at end of file /
    // on error.
    bool next(Bytes &out, size_t &at) {
        if (inf) return next_device(out, at);
        if (at) {
            out.erase_front(at);
            at = 0;
        }
        const size_t CHUNK = 64u << 20;
        for (;;) {
            if (!eof) {
                size_t old = comp.size();
                comp.resize(old + CHUNK);
                size_t got = fread(comp.data() + old, 1, CHUNK, f);
                comp.resize(old + got);
                if (got < CHUNK) eof = true;
            }
            struct Blk { size_t clen, ulen, cdata; };
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
                blks.push_back({bsize - xlen - 20, rd32(comp.data() + p + bsize - 4), p + 12 + xlen});
                p += bsize;
            }
            if (blks.empty()) {
                if (eof) {
                    if (!comp.empty()) err = "truncated BGZF block at end of file";
                    return false;
                }
                continue;   // a single block larger than what was read so far
            }
            std::vector<size_t> uoff(blks.size() + 1, 0);
            for (size_t i = 0; i < blks.size(); i++) uoff[i + 1] = uoff[i] + blks[i].ulen;
            const size_t base = out.size();
            if (!out.resize(base + uoff.back())) { err = "out of host memory"; return false; }
            std::atomic<int> bad{0};
            const Inflater &inf = inflater();
            parallel_for(threads, blks.size() * 4096, [&](size_t b0, size_t b1) {
                if (inf.fast()) {
                    void *d = inf.ld_alloc();
                    if (!d) { bad = 1; return; }
                    for (size_t i = b0 / 4096; i < b1 / 4096; i++) {
                        size_t got = 0;
                        int rc = inf.ld_dec(d, comp.data() + blks[i].cdata, blks[i].clen, out.data() + base + uoff[i],
                                            blks[i].ulen, &got);
                        if (rc != 0 || got != blks[i].ulen) bad = 1;
                    }
                    inf.ld_free(d);
                    return;
                }
                z_stream zs;
                memset(&zs, 0, sizeof zs);
                if (inflateInit2(&zs, -15) != Z_OK) { bad = 1; return; }
                for (size_t i = b0 / 4096; i < b1 / 4096; i++) {
                    inflateReset(&zs);
                    zs.next_in = comp.data() + blks[i].cdata;
                    zs.avail_in = (uInt)blks[i].clen;
                    zs.next_out = out.data() + base + uoff[i];
                    zs.avail_out = (uInt)blks[i].ulen;
                    int rc = inflate(&zs, Z_FINISH);
                    if (rc != Z_STREAM_END || zs.total_out != blks[i].ulen) bad = 1;
                }
                inflateEnd(&zs);
            });
            if (bad) { err = "corrupt BGZF block (inflate failed)"; return false; }
            comp.erase(comp.begin(), comp.begin() + (ptrdiff_t)p);
            return true;
        }
    }
};

// The BAI's linear index (SAM spec 5.2): per contig, the smallest virtual offset of the
// records overlapping each 16 kb window.  Bins are skipped: a coordinate-sorted file read
// from the linear-index offset reaches every record a region query can yield.
struct BaiLinear {
    std::vector<std::vector<uint64_t>> ioff;
    bool load(const std::string &path, std::string &err) {
        FILE *f = fopen(path.c_str(), "rb");
        if (!f) { err = "cannot open BAI: " + path; return false; }
        auto rd = [&](void *p, size_t n) { return fread(p, 1, n, f) == n; };
        char magic[4];
        int32_t n_ref = 0;
        bool ok = rd(magic, 4) && memcmp(magic, "BAI\1", 4) == 0 && rd(&n_ref, 4) && n_ref >= 0;
        if (ok) ioff.resize((size_t)n_ref);
        for (int32_t r = 0; ok && r < n_ref; r++) {
            int32_t n_bin = 0;
            ok = rd(&n_bin, 4) && n_bin >= 0;
            for (int32_t i = 0; ok && i < n_bin; i++) {
                uint32_t bin;
                int32_t n_chunk;
                ok = rd(&bin, 4) && rd(&n_chunk, 4) && n_chunk >= 0 && fseeko(f, 16 * (off_t)n_chunk, SEEK_CUR) == 0;
            }
            int32_t n_intv = 0;
            ok = ok && rd(&n_intv, 4) && n_intv >= 0;
            if (ok) {
                ioff[(size_t)r].resize((size_t)n_intv);
                ok = n_intv == 0 || rd(ioff[(size_t)r].data(), 8 * (size_t)n_intv);
            }
        }
        fclose(f);
        if (!ok) err = "corrupt BAI: " + path;
        return ok;
    }
    // Where a read of the records from (tid, beg) on starts; false = no such record.  A zero
    // entry is a window no record overlapped (older indexers leave those 0 instead of the next
    // window's offset): virtual offset 0 is the BAM header, never a record, so the next
    // non-zero entry -- of this contig or a later one -- is taken instead.
    bool start(int32_t tid, int64_t beg, uint64_t &voff) const {
        for (size_t t = (size_t)std::max(tid, 0); t < ioff.size(); t++) {
            const int64_t w = (int32_t)t == tid ? std::max<int64_t>(beg, 0) >> 14 : 0;
            for (size_t k = (size_t)std::max<int64_t>(w, 0); k < ioff[t].size(); k++)
                if (ioff[t][k] != 0) { voff = ioff[t][k]; return true; }
        }
        return false;
    }
};

// Growable array without value-initialisation; large blocks grow by realloc (mremap on
// glibc), so appending a chunk never re-copies or zero-fills what is already there.
template <typename T>
struct RawVec {
    T *p = nullptr;
    size_t n = 0, cap = 0;
    RawVec() = default;
    RawVec(const RawVec &) = delete;
    RawVec &operator=(const RawVec &) = delete;
    ~RawVec() { free(p); }
    bool resize(size_t m) {
        if (m > cap) {
            size_t c = std::max(m, cap + cap / 2 + 1024);
            T *q = (T *)realloc(p, c * sizeof(T));
            if (!q) return false;
            p = q;
            cap = c;
        }
        n = m;
        return true;
    }
    bool push_back(T v) {
        if (!resize(n + 1)) return false;
        p[n - 1] = v;
        return true;
    }
    size_t size() const { return n; }
    T *data() { return p; }
    const T *data() const { return p; }
    T &operator[](size_t i) { return p[i]; }
    const T &operator[](size_t i) const { return p[i]; }
    void swap(RawVec &o) { std::swap(p, o.p); std::swap(n, o.n); std::swap(cap, o.cap); }
};

}  // namespace

struct svth_bam {
    std::vector<std::string> names;
    std::vector<int64_t> tid_off;
    RawVec<int32_t> pos, endpos;
    RawVec<uint64_t> cig_off;
    RawVec<uint32_t> cigar;
    RawVec<uint8_t> clip;
    int64_t n_records = 0, n_cg = 0;
    double stage_s[6] = {0, 0, 0, 0, 0, 0};   // read, scan, alloc, inflate, wait, total
};

extern "C" {

svth_bam *svth_bam_read(const char *path, int threads, char *err, size_t errcap) {
    return svth_bam_read_region(path, threads, -1, 0, -1, 0, err, errcap);
}

svth_bam *svth_bam_read_region(const char *path, int threads, int32_t tid0, int64_t beg0, int32_t tid1, int64_t end1,
                               char *err, size_t errcap) {
    return svth_bam_read_ex(path, threads, tid0, beg0, tid1, end1, nullptr, err, errcap);
}

svth_bam *svth_bam_read_ex(const char *path, int threads, int32_t tid0, int64_t beg0, int32_t tid1, int64_t end1,
                           const svth_inflater *inf, char *err, size_t errcap) {
    const bool region = tid0 >= 0;
    auto fail = [&](const std::string &m) -> svth_bam * {
        if (err && errcap) snprintf(err, errcap, "%s", m.c_str());
        return nullptr;
    };
    const double t_start = BgzfReader::now();
    FILE *f = fopen(path, "rb");
    if (!f) return fail(std::string("cannot open BAM: ") + path);
    BgzfReader rd;
    rd.f = f;
    rd.threads = threads < 1 ? 1 : threads;
    rd.inf = inf && inf->inflate ? inf : nullptr;
    {
        struct stat st;
        rd.fsize = fstat(fileno(f), &st) == 0 ? (uint64_t)st.st_size : 0;
    }
    Bytes buf;
    size_t at = 0;
    auto need = [&](size_t k) -> bool {
        while (buf.size() - at < k)
            if (!rd.next(buf, at)) return false;
        return true;
    };
    svth_bam *b = new svth_bam();
    auto bail = [&](const std::string &m) {
        rd.drop_pending();   // (the helper thread reads f)
        fclose(f);
        delete b;
        return fail(rd.err.empty() ? m : rd.err);
    };
    // header
    if (!need(8) || memcmp(buf.data() + at, "BAM\1", 4) != 0) return bail("not a BAM file");
    const uint32_t l_text = rd32(buf.data() + at + 4);
    at += 8;
    if (!need((size_t)l_text + 4)) return bail("truncated BAM header");
    at += l_text;
    const int32_t n_ref = (int32_t)rd32(buf.data() + at);
    at += 4;
    if (n_ref < 0) return bail("bad n_ref");
    for (int32_t i = 0; i < n_ref; i++) {
        if (!need(4)) return bail("truncated reference list");
        const uint32_t ln = rd32(buf.data() + at);
        if (!need(4 + (size_t)ln + 4)) return bail("truncated reference list");
        b->names.emplace_back((const char *)buf.data() + at + 4, ln ? ln - 1 : 0);
        at += 4 + ln + 4;
    }
    // region: continue at the BAI's linear-index offset of (tid0, beg0)
    bool done = false;
    if (region) {
        BaiLinear bai;
        std::string e;
        if (!bai.load(std::string(path) + ".bai", e)) return bail(e);
        uint64_t voff = 0;
        if (!bai.start(tid0, beg0, voff)) done = true;   // no record at or after the region start
        else {
            if (!rd.seek(voff >> 16)) return bail("cannot seek in BAM");
            buf.clear();
            at = 0;
            const size_t uo = (size_t)(voff & 0xffff);
            if (uo && !need(uo)) return bail("BAI offset past the end of the BAM");
            at += uo;
        }
    }
    // records, chunk by chunk
    RawVec<int32_t> tid_of;
    std::vector<uint8_t> rec_ok;
    std::vector<uint16_t> flag;
    uint64_t narena = 0;
    std::vector<size_t> roff;
    std::vector<uint32_t> rlen;
    std::vector<bamrec::View> views;
    while (!done) {
        if (buf.size() - at < 4 && !need(4)) break;   // clean EOF
        // sequential boundary scan over the complete records in the buffer
        roff.clear();
        size_t p = at;
        while (buf.size() - p >= 4) {
            const uint32_t bs = rd32(buf.data() + p);
            if (bs < 32) return bail("corrupt BAM record (block_size < 32)");
            if (buf.size() - p < 4 + (size_t)bs) break;
            roff.push_back(p + 4);
            p += 4 + bs;
        }
        if (roff.empty()) {   // one record larger than the buffer: read on
            if (!need(4 + (size_t)rd32(buf.data() + at))) return bail("truncated BAM record");
            continue;
        }
        // pass 1 (parallel): locate every record's CIGAR
        size_t nr = roff.size();
        views.resize(nr);
        parallel_for(rd.threads, nr, [&](size_t i0, size_t i1) {
            for (size_t i = i0; i < i1; i++)
                views[i] = bamrec::view(buf.data() + roff[i], rd32(buf.data() + roff[i] - 4), n_ref);
        });
        if (region)   // sorted file: the first record past (tid1, end1) ends the read
            for (size_t i = 0; i < nr; i++) {
                const int32_t t = (int32_t)rd32(buf.data() + roff[i]), ps = (int32_t)rd32(buf.data() + roff[i] + 4);
                if (t < 0 || t > tid1 || (t == tid1 && (int64_t)ps >= end1)) {
                    nr = i;
                    done = true;
                    p = roff[i] - 4;
                    break;
                }
            }
        // prefix offsets, then pass 2 (parallel): copy into the columnar arrays
        const size_t base = b->pos.size();
        size_t kept = 0;
        for (size_t i = 0; i < nr; i++) {
            if (views[i].bad) return bail("corrupt BAM record");
            if (views[i].ok) kept++;
            if (views[i].cg) b->n_cg++;
        }
        b->n_records += (int64_t)nr;
        std::vector<uint64_t> off(nr + 1, 0);
        std::vector<size_t> slot(nr, 0);
        for (size_t i = 0, k = base; i < nr; i++) {
            off[i + 1] = off[i] + (views[i].ok ? views[i].n : 0);
            slot[i] = views[i].ok ? k++ : (size_t)-1;
        }
        if (!b->pos.resize(base + kept) || !b->endpos.resize(base + kept) || !b->clip.resize(base + kept) ||
            !tid_of.resize(base + kept) || !b->cig_off.resize(base + kept) || !b->cigar.resize(narena + off[nr]))
            return bail("out of host memory");
        parallel_for(rd.threads, nr, [&](size_t i0, size_t i1) {
            for (size_t i = i0; i < i1; i++) {
                const bamrec::View &v = views[i];
                if (!v.ok) continue;
                const size_t k = slot[i];
                uint32_t *dst = b->cigar.data() + narena + off[i];
                if (v.n) memcpy(dst, v.cig, 4ull * v.n);
                b->pos[k] = v.pos;
                b->endpos[k] = bamrec::endpos(v);   // htslib bam_endpos
                b->clip[k] = (uint8_t)v.clip;
                b->cig_off[k] = narena + off[i];
                tid_of[k] = v.tid;
            }
        });
        narena += off[nr];
        at = p;
    }
    rd.drop_pending();
    fclose(f);
    if (!rd.err.empty()) { delete b; return fail(rd.err); }
    {
        const double st[6] = {rd.t_read, rd.t_scan, rd.t_alloc_r + rd.t_alloc, rd.t_inflate, rd.t_wait,
                              BgzfReader::now() - t_start};
        memcpy(b->stage_s, st, sizeof st);
    }
    const size_t n = b->pos.size();
    if (!b->cig_off.push_back(narena)) { delete b; return fail("out of host memory"); }
    // per-tid ranges; reorder only when the file was not coordinate-sorted
    bool sorted = true;
    for (size_t i = 1; i < n && sorted; i++)
        sorted = tid_of[i] > tid_of[i - 1] || (tid_of[i] == tid_of[i - 1] && b->pos[i] >= b->pos[i - 1]);
    if (!sorted) {
        std::vector<size_t> idx(n);
        std::iota(idx.begin(), idx.end(), 0);
        std::stable_sort(idx.begin(), idx.end(), [&](size_t x, size_t y) {
            return tid_of[x] != tid_of[y] ? tid_of[x] < tid_of[y] : b->pos[x] < b->pos[y];
        });
        RawVec<int32_t> pos2, end2, tid2;
        RawVec<uint8_t> clip2;
        RawVec<uint64_t> off2;
        RawVec<uint32_t> cig2;
        if (!pos2.resize(n) || !end2.resize(n) || !tid2.resize(n) || !clip2.resize(n) || !off2.resize(n + 1) ||
            !cig2.resize(narena)) { delete b; return fail("out of host memory"); }
        uint64_t w = 0;
        for (size_t k = 0; k < n; k++) {
            const size_t i = idx[k];
            pos2[k] = b->pos[i]; end2[k] = b->endpos[i]; clip2[k] = b->clip[i]; tid2[k] = tid_of[i];
            const uint64_t o = b->cig_off[i], m = b->cig_off[i + 1] - o;
            off2[k] = w;
            if (m) memcpy(cig2.data() + w, b->cigar.data() + o, 4 * m);
            w += m;
        }
        off2[n] = w;
        b->pos.swap(pos2); b->endpos.swap(end2); b->clip.swap(clip2); b->cig_off.swap(off2); b->cigar.swap(cig2);
        tid_of.swap(tid2);
    }
    b->tid_off.assign((size_t)n_ref + 1, 0);
    for (size_t k = 0; k < n; k++) b->tid_off[(size_t)tid_of[k] + 1]++;
    for (int32_t t = 0; t < n_ref; t++) b->tid_off[(size_t)t + 1] += b->tid_off[(size_t)t];
    return b;
}

int svth_bam_read_device(const char *path, int threads, const svth_dev_sink *sink, int32_t *n_targets, double *stage4,
                         char *err, size_t errcap) {
    auto fail = [&](const std::string &m) {
        if (err && errcap) snprintf(err, errcap, "%s", m.c_str());
        return 1;
    };
    if (!sink || !sink->begin || !sink->feed) return fail("no device sink");
    const double t_start = BgzfReader::now();
    FILE *f = fopen(path, "rb");
    if (!f) return fail(std::string("cannot open BAM: ") + path);
    BgzfReader rd;
    rd.f = f;
    rd.threads = threads < 1 ? 1 : threads;
    // batches of whole BGZF blocks through read_next (its input buffers from the sink's allocator)
    svth_inflater cfg{};
    cfg.alloc = sink->alloc;
    cfg.release = sink->release;
    cfg.user = sink->user;
    cfg.batch_bytes = sink->batch_bytes;
    rd.inf = &cfg;
    {
        struct stat st;
        rd.fsize = fstat(fileno(f), &st) == 0 ? (uint64_t)st.st_size : 0;
    }
    auto bail = [&](const std::string &m) {
        rd.drop_pending();
        fclose(f);
        return fail(rd.err.empty() ? m : rd.err);
    };
    BgzfReader::Comp c = rd.read_next();
    if (!c.ok) return bail(c.err);
    if (c.blks.empty()) return bail("not a BAM file (no BGZF blocks)");
    // the header (magic, text, references) on the host: inflate the first blocks until it is complete
    std::vector<uint8_t> h;
    size_t bi = 0;
    auto need = [&](size_t k) -> bool {
        while (h.size() < k) {
            if (bi >= c.blks.size()) return false;
            const svt_bgzf_block &b = c.blks[bi++];
            const size_t o = h.size();
            h.resize(o + b.ulen);
            z_stream zs;
            memset(&zs, 0, sizeof zs);
            if (inflateInit2(&zs, -15) != Z_OK) return false;
            zs.next_in = rd.cins[c.i].p + b.coff;
            zs.avail_in = (uInt)b.clen;
            zs.next_out = h.data() + o;
            zs.avail_out = (uInt)b.ulen;
            const int rc = inflate(&zs, Z_FINISH);
            inflateEnd(&zs);
            if (rc != Z_STREAM_END || zs.total_out != b.ulen) return false;
        }
        return true;
    };
    if (!need(8) || memcmp(h.data(), "BAM\1", 4) != 0) return bail("not a BAM file");
    size_t at = 8 + (size_t)rd32(h.data() + 4);
    if (!need(at + 4)) return bail("truncated BAM header (or longer than one batch)");
    const int32_t n_ref = (int32_t)rd32(h.data() + at);
    at += 4;
    if (n_ref < 0) return bail("bad n_ref");
    for (int32_t i = 0; i < n_ref; i++) {
        if (!need(at + 4)) return bail("truncated reference list (or longer than one batch)");
        const uint32_t ln = rd32(h.data() + at);
        at += 4 + (size_t)ln + 4;
        if (!need(at)) return bail("truncated reference list (or longer than one batch)");
    }
    if (n_targets) *n_targets = n_ref;
    char e[512] = {0};
    if (sink->begin(sink->user, n_ref, e, sizeof e) != 0) return bail(e[0] ? e : "device sink: begin failed");
    // the batches: the next one read and scanned by a helper thread while this one is decoded
    double t_feed = 0, t_wait = 0;
    uint64_t skip = at;
    for (;;) {
        if (!rd.eof || rd.carry_n) rd.pending_comp = std::async(std::launch::async, [&rd] { return rd.read_next(); });
        const double t0 = BgzfReader::now();
        const int rc = sink->feed(sink->user, rd.cins[c.i].p, c.p, c.blks.data(), c.blks.size(), skip, e, sizeof e);
        t_feed += BgzfReader::now() - t0;
        skip = 0;
        if (rc != 0) return bail(e[0] ? e : "device sink: feed failed");
        if (!rd.pending_comp.valid()) break;
        const double t1 = BgzfReader::now();
        c = rd.pending_comp.get();
        t_wait += BgzfReader::now() - t1;
        if (!c.ok) return bail(c.err);
        if (c.blks.empty()) break;
    }
    rd.drop_pending();
    fclose(f);
    if (stage4) {
        stage4[0] = rd.t_read;
        stage4[1] = t_feed;
        stage4[2] = t_wait + rd.t_alloc_r;
        stage4[3] = BgzfReader::now() - t_start;
    }
    return 0;
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
void svth_bam_stage_seconds(const svth_bam *b, double *s6) { memcpy(s6, b->stage_s, sizeof b->stage_s); }

}  // extern "C"
