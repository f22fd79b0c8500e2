// svt_engine.hip -- MI355X (gfx950) SV-refinement engine: HIP kernels + the C ABI of
// include/svtrek_gpu.h.
//
// One wavefront (one 64-lane workgroup) per query WINDOW (a DEL locus has two: the
// refine_start and refine_end windows; an INS locus one).  Per window the wave
//   1. finds the yielded read range [lo, hi) of htslib's region query (A3) with a
//      bucket index (first read per 4 kb of contig) + one 64-lane probe each for the
//      sorted pos[] and the prefix-max-of-endpos emax[] arrays;
//   2. streams the window's CIGAR words -- the reads [lo, hi) own ONE contiguous span
//      of the CIGAR arena -- in 1024-op tiles, four 16-B loads per lane (4 KiB per wave,
//      fully coalesced, next tile prefetched while the current one is processed).  A segmented wave prefix scan (DPP) of the reference advance, reset at
//      each read's first op to its pos, gives every op's walk position at once; because
//      the walk position only grows inside a read, "this op comes after the break of
//      refinement.c:141-144" is just `position before the op > inter.end`, so no second
//      scan is needed.  Breakpoint candidates (A4-A6) and the soft-clip candidates of
//      each read's stop op are appended to LDS with LDS atomics; tails of reads that
//      already broke (and reads that do not overlap the window) are skipped;
//   3. bitonic-sorts the candidates in LDS and runs consensus_pos's asymmetric vote
//      (A8-A10): per-element cluster counts in parallel (binary search + int64 prefix
//      sums), the greedy accept with scalar readlanes.
// Windows with more than SVT_LDS_CANDS candidates re-run on a slab of a device spill
// pool (exact).  Reads whose walk could wrap uint32 go through a per-read wave walk
// (walk_read) that replays the reference's uint32 arithmetic op by op.  No floating
// point, no MFMA: integer scan + vote, HBM-streaming bound.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <new>
#include <atomic>
#include <type_traits>
#include <thread>
#include <vector>

#include "../../include/svtrek_gpu.h"
#include "svt_bamrec.h"

#define SVT_VERSION "svtrek_amd 0.25.0 (gfx950, value-bucketed event index filed by a lane-per-read walk with a 9-B LDS stage, band + prefix-max facts, packed span walk fed by readlane, lane vote, BGZF inflate + BAM decode)"

namespace {

constexpr int WAVE = 64;
constexpr int CAP = SVT_LDS_CANDS;          // LDS candidates per window
constexpr int SV_MIN_LENGTH = 50;           // params.h:33
constexpr uint32_t OP_INS = 1, OP_DEL = 2, OP_SOFT = 4;   // params.h:11-14
constexpr int K_START = 0, K_END = 1, K_INS = 2;          // refine_start / refine_end / refine_ins
constexpr int32_t T_INS = 1, T_DEL = 2;
constexpr int BKT_SHIFT = 12;               // read-start bucket = 4096 bp
constexpr uint32_t NCIG_MASK = 0x1fffffffu; // rec.z: n_cigar | clip << 30
constexpr uint32_t STREAM_PAD = 4096;       // zero words after the CIGAR stream (the index walks' slot over-read)
// Walk positions in the index saturate at IX_SAT.  The reference's uint32 reference_pos
// (refinement.c:118-145) cannot wrap before it passes a window end below 2^30 (one op
// advances it by < 2^28), so for every window with e < WEXACT "walk position <= e" and every
// candidate value are exact on saturated positions; windows ending at or past WEXACT take the
// per-read replay of the reference's uint32 arithmetic (walk_read).
constexpr uint32_t IX_SAT = 1u << 30;
constexpr uint32_t WEXACT = 1u << 30;
// Span events (svt_load_pileup, the index builds): every read's breakpoint events, 16 B each,
// self-contained {x, w, endpos, aux} so that a window is one filter over a contiguous span:
//   D list: D > 50 ops {walk position before the op, CIGAR word, endpos, 0} (refinement.c:124,:188),
//           SP_TRAIL {walk end, SP_TRAIL, endpos, 0} for cigar[n-1] == S (:120,:147),
//           SP_LEAD {pos, SP_LEAD, endpos, walk end} for cigar[0] == S (:210);
//   I list: I >= 50 ops {walk position before the op, CIGAR word, endpos, 0} (refinement.c:299).
constexpr uint32_t SP_TRAIL = 0xEu, SP_LEAD = 0xFu;   // op codes no candidate event carries

struct DevPileup {
    const int32_t *pos;       // [n_reads]
    const int32_t *emax;      // [n_reads] prefix max of endpos within the contig
    const uint4 *rec;         // [n_reads] {pos, endpos, n_cig | clip<<30, 0}
    const uint64_t *off64;    // [n_reads+1] read r's CIGAR = cigar[off64[r] .. off64[r] + n_cig)
    const int64_t *tid_off;   // [n_targets+1]
    const int64_t *bkt_off;   // [n_targets+1] start of each contig's bucket table
    const uint2 *bkt;         // {first read with pos >= b << BKT_SHIFT, first read with emax >= b << BKT_SHIFT}
    const uint32_t *cigar;    // the CIGAR stream (caller's words; one 0M word for n_cigar == 0 reads)
    const uint64_t *spoffD;   // [n_reads+1] span events: read r's D-list events are spD[spoffD[r] .. spoffD[r+1])
    const uint64_t *spoffI;   // [n_reads+1]              its I-list events spI[spoffI[r] .. spoffI[r+1])
                              // (= the I >= 50 ops before read r: the POA mode's sequence index)
    const uint4 *spD;
    const uint4 *spI;
    int32_t n_targets;
};

// The value-bucketed event index (svt_bucket.inc, svt_bucket_build.inc): per window kind one array
// of events filed by candidate value in 1 kb buckets per contig.
constexpr int BKS = 10;                                  // bucket = 1 kb of candidate value
constexpr int BA_S = 0, BA_E = 1, BA_I = 2, BA_L = 3, BA_N = 4;
struct BkIndex {
    const uint4 *ev;              // the events of the four arrays, S, E, I, L one after the other -- S: D > 50
                                  // + trailing S by x; E: D > 50 by x + len + 1, leading S by walk end + 1;
                                  // I: I >= 50 by x; L: leading S by read start
    const uint32_t *off;          // [BA_N][nbk + 1] first event (an index into ev) of every bucket
    const int32_t *pm;            // [3][nbk + 1] S, E, I: prefix max (within the contig) of the BELOW keys
    const uint64_t *cbase;        // [n_targets] contig t's first bucket
    const uint32_t *cnb;          // [n_targets] its buckets (the last one: every value past the others)
    const uint32_t *maxd;         // [n_targets] its longest D > 50 op (0: none)
    uint64_t nbk;                 // buckets per array (every contig's)
    int on;                       // built (SVTREK_INDEX=lists: 0, the span lists alone)
};

struct KParams {
    int32_t wider, median, narrow, range, ci, min_count;
    int32_t sw_window, sw_slide;   // sliding_window_ins mode only
    // refine_end's leading-S reads whose walk passes e (refinement.c:210-221) push the position
    // after the break op + 1 >= e + 2.  When e + 2 already lies at or past everything the vote
    // reads -- pos + range + max(ci, 0) and pos + 26 (narrow + 2 >= both widths) -- any value
    // >= e + 2 votes the same (see band_filter), so these reads count as one candidate at e + 2
    // and no stop search is needed; otherwise refine_end windows take the per-read replay.
    int32_t sent_ok;
};

struct KArgs {
    DevPileup pile;
    KParams prm;
    const svt_locus *loci;
    svt_result *out;
    uint32_t n;                 // loci
    int32_t *pool;              // spill slabs (int32 words)
    unsigned long long *pool_head;   // epoch << 40 | words handed out in that launch
    unsigned long long pool_words;
    uint32_t epoch;                  // this launch's pool epoch (1 .. 2^24-1)
    int32_t *status;            // bit0: spill pool exhausted
    unsigned long long *work;   // svt_work counters (COUNT builds only)
    const uint4 *sw_sub;        // sliding_window_ins mode: per sub-window {chrom, start, end, 0}
    int2 *sw_out;               //   per sub-window {bestCandidate, maxSupport}
    uint4 *rec_out;             // gather records {index, start, end, 0} instead of `out` (or null)
    const uint32_t *rec_index;  //   index of locus i: rec_index[i], or rec_base + i when null
    uint32_t rec_base;
    uint32_t *redo_list;        // lane-vote launches: windows left for refine_redo_kernel
    uint32_t *redo_ctr;         //   their count (this launch's counter)
    uint32_t *redo_next;        //   the next launch's counter (reset by refine_redo_kernel)
    BkIndex bk;                 // the value-bucketed event index
};

// svt_work counter slots (refine_window's wk[], the context's work words)
constexpr int W_WINDOWS = 0, W_READS = 1, W_OPS = 2, W_CANDS = 3, W_SPILLED = 4, W_QUERIES = 5, W_PROBE = 6,
              W_RANGE = 7, W_LREADS = 8, W_LENTRIES = 9, W_STOPS = 10, W_STOPCH = 11, W_SQUERIES = 12,
              W_SPAN = 13, W_BQ = 14, W_BEV = 15, W_N = 16;
constexpr size_t CTL_BYTES = 256;   // context control words: pool head, status, work counters
constexpr size_t CTL_REDO = 200;    // redo counters: two alternating (direct launches), one + scratch (captured)
static_assert(16 + 8 * W_N <= CTL_REDO && CTL_REDO + 16 <= CTL_BYTES, "control block too small");

// ------------------------------------------------------------------ wave primitives
#define SVT_COLD __forceinline__   // (cold paths inlined: out-of-line calls measured slower)
__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }
// The lane mask of p straight from its compare (no v_cndmask / v_cmp round trip through a VGPR).
__device__ __forceinline__ uint64_t ballot(bool p) { return (uint64_t)__builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ uint32_t rdlane(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ int32_t rdlane_i(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t rdlane64(uint64_t v, int l) {
    uint32_t lo = rdlane((uint32_t)v, l), hi = rdlane((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ int32_t uniform_i(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }
// Every window is owned by ONE wave (several independent waves share a workgroup), so the
// only ordering ever needed is between the lanes of a wave: a workgroup-scope
// release/acquire pair around a wave barrier (no s_barrier across the workgroup).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWMASK, 0xf, false);
}
template <int CTRL, int ROWMASK>
__device__ __forceinline__ int32_t dpp_i(int32_t v, int32_t identity) {
    return __builtin_amdgcn_update_dpp(identity, v, CTRL, ROWMASK, 0xf, false);
}
// DPP controls (GFX9): row_shr:n = 0x110+n, wave_shr:1 = 0x138, row_bcast:15 = 0x142, row_bcast:31 = 0x143

// Inclusive wave64 prefix sum (mod 2^32).
__device__ __forceinline__ uint32_t wave_scan_add(uint32_t v) {
    v += dpp<0x111, 0xf>(v);
    v += dpp<0x112, 0xf>(v);
    v += dpp<0x114, 0xf>(v);
    v += dpp<0x118, 0xf>(v);
    v += dpp<0x142, 0xa>(v);
    v += dpp<0x143, 0xc>(v);
    return v;
}

// Inclusive wave64 max scan (identity -1).
__device__ __forceinline__ int32_t wave_scan_max(int32_t v) {
    v = max(v, dpp_i<0x111, 0xf>(v, -1));
    v = max(v, dpp_i<0x112, 0xf>(v, -1));
    v = max(v, dpp_i<0x114, 0xf>(v, -1));
    v = max(v, dpp_i<0x118, 0xf>(v, -1));
    v = max(v, dpp_i<0x142, 0xa>(v, -1));
    v = max(v, dpp_i<0x143, 0xc>(v, -1));
    return v;
}

__device__ __forceinline__ int64_t wave_scan_add64(int64_t x) {
    int l = lane_id();
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
        int64_t y = __shfl_up(x, (unsigned)d, WAVE);
        if (l >= d) x += y;
    }
    return x;
}

// First index in [l, h) whose key satisfies pred (pred monotone false..true), 64-ary.
template <typename Pred>
__device__ SVT_COLD int64_t wave_partition_point(int64_t l, int64_t h, Pred pred) {   // cold: > 64 reads per bucket
    const int ln = lane_id();
    while (h - l > WAVE) {
        int64_t span = h - l;
        int64_t p = l + ((int64_t)(ln + 1) * span) / (WAVE + 1);
        uint64_t m = ballot(pred(p));
        int k = m ? __builtin_ctzll(m) : WAVE;
        int64_t nl = k == 0 ? l : l + ((int64_t)k * span) / (WAVE + 1) + 1;
        int64_t nh = k == WAVE ? h : l + ((int64_t)(k + 1) * span) / (WAVE + 1) + 1;
        l = nl;
        h = nh < h ? nh : h;
    }
    int64_t p = l + ln;
    uint64_t m = ballot(p < h && pred(p));
    return m ? l + __builtin_ctzll(m) : h;
}

// ------------------------------------------------------------------ candidate sink
// Candidates are appended with LDS atomics: their order is irrelevant (the multiset is
// sorted before the vote) and they are rare next to the CIGAR ops streamed, so a lane
// that finds one appends it on its own, under any divergence.
struct Sink {
    int32_t *buf;   // LDS or a global spill slab
    int32_t cap;
    int32_t *cnt;   // LDS counter: candidates seen (may exceed cap -> spill re-run)
    __device__ __forceinline__ void push1(int32_t val) {
        int idx = atomicAdd(cnt, 1);
        if (idx < cap) buf[idx] = val;
    }
    __device__ __forceinline__ void push(bool pred, int32_t val) {
        if (pred) push1(val);
    }
};

struct WinStats {
    unsigned long long reads = 0, ops = 0;
    // span walk's own reads (svt_count_work): see svt_work
    unsigned long long queries = 0, probe = 0, range = 0, lreads = 0, lentries = 0, stops = 0, stopch = 0;
    unsigned long long squeries = 0, span = 0;   // span walk (G_SPAN COUNT builds)
};

template <int KIND>
__device__ __forceinline__ bool is_candidate_op(uint32_t op, uint32_t len) {
    if (KIND == K_INS) return op == OP_INS && (uint32_t)SV_MIN_LENGTH <= len;   // refinement.c:299
    return op == OP_DEL && (uint32_t)SV_MIN_LENGTH < len;                       // refinement.c:124,:188
}

// Per-read walk, 64 ops per step, replaying the reference's uint32 position arithmetic
// exactly (refinement.c:118-159 / :184-221 / :295-318).  Used for reads whose walk could
// wrap 2^32 (never in practice) and by the per-read gather variant.
template <int KIND, bool COUNT>
__device__ __forceinline__ void walk_read(const uint32_t *__restrict__ cigar, uint64_t off, uint32_t n, uint32_t rpos,
                          uint32_t clip, uint32_t s, uint32_t e, Sink &sink, WinStats &st) {
    const int ln = lane_id();
    uint32_t carry = rpos;
    bool broke = false;
    uint32_t stop_rp = 0;
    uint32_t walked = n;
    for (uint32_t cb = 0; cb < n; cb += WAVE) {
        uint32_t i = cb + (uint32_t)ln;
        bool v = i < n;
        uint32_t w = v ? cigar[off + i] : 0u;
        uint32_t op = w & 0xfu, len = w >> 4;
        uint32_t adv = (op != OP_INS && op != OP_SOFT) ? len : 0u;   // refinement.c:141
        uint32_t after = carry + wave_scan_add(adv);
        uint32_t before = after - adv;
        uint64_t bm = ballot(v && after > e);                         // refinement.c:145
        int fb = bm ? __builtin_ctzll(bm) : WAVE;
        bool hit = v && ln <= fb && is_candidate_op<KIND>(op, len);
        sink.push(hit, KIND == K_END ? (int32_t)(before + len + 1u) : (int32_t)before);   // :198 / :134
        if (bm) {
            broke = true;
            stop_rp = rdlane(after, fb);
            walked = cb + (uint32_t)fb + 1u;
            break;
        }
        carry = rdlane(after, WAVE - 1);
    }
    if (KIND == K_START) {   // trailing soft clip, refinement.c:120,:147-159
        bool c = (clip & SVT_CLIP_LAST_S) && !broke && s <= carry && carry <= e;
        sink.push(c && ln == 0, (int32_t)carry);
    } else if (KIND == K_END) {   // leading soft clip, refinement.c:210-221 (rp = walked position)
        bool c = (clip & SVT_CLIP_FIRST_S) && (int64_t)s <= (int64_t)(int32_t)rpos &&
                 (int64_t)(int32_t)rpos <= (int64_t)e;
        sink.push(c && ln == 0, (int32_t)((broke ? stop_rp : carry) + 1u));
    }
    if (COUNT) {
        st.reads++;
        uint64_t wk = walked;
        if (KIND == K_START && (n == 0 || (broke && walked < n))) wk++;   // cigar[n-1] test
        if (KIND == K_END && n == 0) wk++;                                 // cigar[0] test
        st.ops += wk;
    }
}

// ------------------------------------------------------------------ read range (A3)
// sam_itr_queryi(idx, chrom-1, inter.start-1, inter.end-1) (refinement.c:114): the reads
// [lo, hi) of contig tid may overlap [beg, end) (each still needs endpos > beg), with
//   hi = first read with pos >= end,  lo = first read with emax > beg  (emax = prefix max
//   of endpos, so every read before lo ends at or before beg).
// The bucket table gives, per 4 kb bucket b, {first read with pos >= b*4096, first read with
// emax >= b*4096}; each bound then lies inside one bucket, and the two searches share two
// dependent steps: 4 bucket words, then one 64-lane probe each of pos[] and emax[].
__device__ __forceinline__ int64_t probe_first(int64_t l, int64_t h, bool hit_in_lane, bool lane_valid) {
    const uint64_t m = ballot(lane_valid && hit_in_lane);
    return m ? l + __builtin_ctzll(m) : h;
}

__device__ __forceinline__ bool read_range(const DevPileup &P, int tid, int64_t beg, int64_t end, int64_t &lo,
                                           int64_t &hi, WinStats *st = nullptr) {
    if (tid < 0 || tid >= P.n_targets || end <= beg) return false;   // no reads (A3)
    const int64_t ra = P.tid_off[tid], nr = P.tid_off[tid + 1] - ra;
    if (nr == 0) return false;
    const int64_t b0 = P.bkt_off[tid], nb = P.bkt_off[tid + 1] - b0;   // last bucket = {nr, nr}
    const int ln = lane_id();
    const int64_t bi = min((ln < 2 ? end >> BKT_SHIFT : beg >> BKT_SHIFT) + (ln & 1), nb - 1);
    const uint2 bw = ln < 4 ? P.bkt[b0 + bi] : make_uint2(0, 0);
    const int64_t hl = rdlane(bw.x, 0), hh = rdlane(bw.x, 1), ll = rdlane(bw.y, 2), lh = rdlane(bw.y, 3);
    const int32_t *pos = P.pos + ra, *emax = P.emax + ra;
    const bool vh = hl + ln < hh, vl = ll + ln < lh;
    const int32_t pv = vh ? pos[hl + ln] : 0, ev = vl ? emax[ll + ln] : 0;
    int64_t h = probe_first(hl, hh, (int64_t)pv >= end, vh);
    int64_t l = probe_first(ll, lh, (int64_t)ev > beg, vl);
    if (hh - hl > WAVE) h = wave_partition_point(hl, hh, [&](int64_t r) { return (int64_t)pos[r] >= end; });
    if (lh - ll > WAVE) l = wave_partition_point(ll, lh, [&](int64_t r) { return (int64_t)emax[r] > beg; });
    if (st) {   // COUNT builds: the bucket words + each search's entries up to its boundary
        st->queries++;
        st->probe += (unsigned long long)((h - hl) + (h < hh ? 1 : 0) + (l - ll) + (l < lh ? 1 : 0));
    }
    lo = ra + l;
    hi = ra + h;
    return lo < hi;
}

// ------------------------------------------------------------------ per-read gather (v1)
template <int KIND, bool COUNT>
__device__ __forceinline__ void gather_perread(const DevPileup &P, int tid, uint32_t s, uint32_t e, Sink &sink, WinStats &st) {
    const int64_t beg = (int64_t)(uint32_t)(s - 1u), end = (int64_t)(uint32_t)(e - 1u);
    int64_t lo, hi;
    if (!read_range(P, tid, beg, end, lo, hi)) return;
    const int ln = lane_id();
    for (int64_t base = lo; base < hi; base += WAVE) {
        int64_t r = base + ln;
        bool valid = r < hi;
        uint4 rc = valid ? P.rec[r] : make_uint4(0, 0, 0, 0);
        bool ov = valid && (int64_t)(int32_t)rc.y > beg;   // pos < end holds below hi (hts_itr_next)
        uint64_t m = ballot(ov);
        while (m) {
            int l = __builtin_ctzll(m);
            m &= m - 1;
            uint32_t z = rdlane(rc.z, l);
            walk_read<KIND, COUNT>(P.cigar, P.off64[base + l], z & NCIG_MASK, rdlane(rc.x, l), z >> 30, s, e, sink,
                                   st);
        }
    }
}

// ------------------------------------------------------------------ shared helpers
__device__ __forceinline__ uint32_t ref_adv(uint32_t w) {   // refinement.c:141: every op but I (1) and S (4)
    return (w >> 4) & (uint32_t)__builtin_amdgcn_sbfe((int)~0x12u, w & 0xfu, 1);
}

#ifndef SVT_VOTE2
#define SVT_VOTE2 0              // 1: a window's two vote passes in two lanes (parity-green, no faster: profiles/r06_AA)
#endif
#ifndef SVT_DIAG
#define SVT_DIAG 0               // diagnostic builds only (wrong results): 1 = region query only, 3 = no refine_end
                                 // stop search, 4 = no sort/vote, 5 = sort + prefix sums, no vote, ...,
                                 // 23 = the lane emit without its CIGAR walk (svt_index2.inc, profiles/r05_AK)
#endif


// ------------------------------------------------------------------ span walk (default)
// The reads [lo, hi) of a window own one contiguous span of the D (or I) event list, and
// every event carries what its tests need (its read's endpos for the overlap test of
// hts_itr_next), so a window is: region query, the span's two bounds, then ONE filter over
// the span, every load of a 256-event batch issued at once (no per-read dependent chain).
// An op is processed by the reference walk iff the walk position before it is <= inter.end
// (positions only grow along a read, refinement.c:145), so a candidate event counts iff
// x <= e; the soft-clip events follow refinement.c:147-159 (trailing S: no break, s <= walk
// end <= e) and :210-220 (leading S, s <= pos <= e: walk end + 1, or -- the walk passes e --
// the position after the break op + 1, which votes as e + 2: KParams::sent_ok).
constexpr int SPAN_U = 4;   // 16-B event loads in flight per lane

__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// The span walk's own reads, for svt_count_work: the region query and the events of the span.
template <int KIND>
__device__ __forceinline__ void span_count(const DevPileup &P, int tid, uint32_t s, uint32_t e, WinStats &st) {
    const int64_t beg = (int64_t)(uint32_t)(s - 1u), end = (int64_t)(uint32_t)(e - 1u);
    int64_t lo, hi;
    if (!read_range(P, tid, beg, end, lo, hi, &st)) return;
    const uint64_t *off = KIND == K_INS ? P.spoffI : P.spoffD;
    st.squeries++;
    st.span += off[hi] - off[lo];
}

// read_range (A3) with the span bounds read in the same dependent step as the pos/emax
// probes: each probe lane also loads the span offset of its read, and the bounds are taken
// from the lanes where the two searches end (one HBM round trip less per window).  Wider
// bucket ranges fall back to read_range + one more step.
template <int KIND>
__device__ __forceinline__ bool span_query(const DevPileup &P, int tid, int64_t beg, int64_t end, uint64_t &E0,
                                           uint64_t &E1) {
    if (tid < 0 || tid >= P.n_targets || end <= beg) return false;   // no reads (A3)
    const int64_t ra = P.tid_off[tid], nr = P.tid_off[tid + 1] - ra;
    if (nr == 0) return false;
    const uint64_t *off = KIND == K_INS ? P.spoffI : P.spoffD;
    const int64_t b0 = P.bkt_off[tid], nb = P.bkt_off[tid + 1] - b0;   // last bucket = {nr, nr}
    const int ln = lane_id();
    const int64_t bi = min((ln < 2 ? end >> BKT_SHIFT : beg >> BKT_SHIFT) + (ln & 1), nb - 1);
    const uint2 bw = ln < 4 ? P.bkt[b0 + bi] : make_uint2(0, 0);
    const int64_t hl = rdlane(bw.x, 0), hh = rdlane(bw.x, 1), ll = rdlane(bw.y, 2), lh = rdlane(bw.y, 3);
    if (hh - hl >= WAVE || lh - ll >= WAVE) {   // wide bucket: the general search, then the bounds
        int64_t lo, hi;
        if (!read_range(P, tid, beg, end, lo, hi)) return false;
        const uint64_t ob = ln < 2 ? off[ln ? hi : lo] : 0ull;
        E0 = rdlane64(ob, 0);
        E1 = rdlane64(ob, 1);
        return true;
    }
    // lanes [0, hh-hl] cover the hi candidates hl .. hh, lanes [0, lh-ll] the lo candidates
    const bool vh = hl + ln <= hh, vl = ll + ln <= lh;
    const int64_t rh = ra + (vh ? hl + ln : hl), rl = ra + (vl ? ll + ln : ll);
    const int32_t pv = vh && hl + ln < hh ? P.pos[rh] : 0, ev = vl && ll + ln < lh ? P.emax[rl] : 0;
    const uint64_t oh = off[rh], ol = off[rl];
    const uint64_t mh = ballot(vh && hl + ln < hh && (int64_t)pv >= end);
    const uint64_t ml = ballot(vl && ll + ln < lh && (int64_t)ev > beg);
    const int kh = mh ? __builtin_ctzll(mh) : (int)(hh - hl), kl = ml ? __builtin_ctzll(ml) : (int)(lh - ll);
    if (ll + kl >= hl + kh) return false;
    E1 = rdlane64(oh, kh);
    E0 = rdlane64(ol, kl);
    return true;
}

// One span event's test for window [s, e] (query beg = s-1): it is a candidate with value val.
// A leading-S read whose walk passes e (refine_end's stop, :210-221) is one at e + 2.
template <int KIND>
__device__ __forceinline__ bool span_cand(const uint4 &v, uint32_t s, uint32_t e, int32_t beg32, uint32_t &val) {
    const uint32_t x = v.x, op = v.y & 0xfu, len = v.y >> 4;
    const bool ovl = (int32_t)v.z > beg32;   // hts_itr_next overlap; pos < end holds below hi
    val = x;
    if (KIND == K_INS) return ovl && op == OP_INS && x <= e;                   // refinement.c:299
    if (KIND == K_START) return ovl && x <= e && (op == OP_DEL || (op == SP_TRAIL && s <= x));   // :124 / :147-159
    const bool lead = op == SP_LEAD && ovl && s <= x && x <= e;                // :210-220
    val = op == OP_DEL ? x + len + 1u : v.w > e ? e + 2u : v.w + 1u;
    return (ovl && x <= e && op == OP_DEL) || lead;                            // :188-199
}

template <int KIND>
__device__ __forceinline__ void span_walk(const DevPileup &P, uint32_t s, uint32_t e, uint64_t E0, uint64_t E1,
                                          Sink &sink) {
    const int32_t beg32 = (int32_t)(uint32_t)(s - 1u);   // yielded reads: beg < end <= 2^30
    const int ln = lane_id();
    const uint4 *ev = KIND == K_INS ? P.spI : P.spD;
    int32_t cnt = 0;   // candidates appended so far (wave-uniform)
    for (uint64_t b = E0; b < E1; b += SPAN_U * WAVE) {
        uint4 v[SPAN_U];
        const uint64_t left = E1 - b;   // events from b on (wave-uniform): the u-slots past them are skipped
        // loads with clamped indices and no branches, so that all of them are in flight
        // before the first is used; lanes past E1 are masked below
#pragma unroll
        for (int u = 0; u < SPAN_U; u++) {
            const uint64_t j = b + (uint64_t)(u * WAVE + ln);
            if ((uint64_t)(u * WAVE) < left) v[u] = ev[j < E1 ? j : E1 - 1];
        }
#pragma unroll
        for (int u = 0; u < SPAN_U; u++) {
            if ((uint64_t)(u * WAVE) >= left) break;
            if ((uint64_t)(u * WAVE + ln) >= left) v[u] = make_uint4(0, 0, 0, 0);   // zero event: no candidate
            uint32_t val;
            const bool c = span_cand<KIND>(v[u], s, e, beg32, val);
            const uint64_t m = ballot(c);
            const int32_t idx = cnt + (int32_t)mbcnt(m);
            if (c && idx < sink.cap) sink.buf[idx] = (int32_t)val;
            cnt += (int32_t)__popcll(m);
        }
    }
    if (ln == 0) *sink.cnt = cnt;
}

// The wave-wide gather of one window: the span walk, or the reference's own per-read walk for
// windows ending at or past WEXACT and for refine_end windows whose leading-S stops cannot
// vote as e + 2 (!sent_ok).
template <int KIND, bool COUNT>
__device__ __forceinline__ void gather_span(const DevPileup &P, const KParams &k, int tid, uint32_t s, uint32_t e,
                                            Sink &sink, WinStats &st) {
    if (COUNT) {   // diagnostic: the reference's work by the exact per-read walk + what the span walk reads
        gather_perread<KIND, true>(P, tid, s, e, sink, st);
        if (e < WEXACT) span_count<KIND>(P, tid, s, e, st);
        return;
    }
    if (e >= WEXACT || (KIND == K_END && !k.sent_ok)) { gather_perread<KIND, COUNT>(P, tid, s, e, sink, st); return; }
    const int64_t beg = (int64_t)(uint32_t)(s - 1u), end = (int64_t)(uint32_t)(e - 1u);
    uint64_t E0, E1;
    if (!span_query<KIND>(P, tid, beg, end, E0, E1)) return;
#if SVT_DIAG == 1
    return;     // diagnostic build: region query only
#endif
    span_walk<KIND>(P, s, e, E0, E1, sink);
}

// ------------------------------------------------------------------ sort + vote (A8-A10)
// Bitonic sort of buf[0..N) (N power of two, padded with INT32_MAX) by one wave.
__device__ __forceinline__ void wave_bitonic_sort(int32_t *buf, int N) {
    const int ln = lane_id();
    for (int k = 2; k <= N; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = ln; i < N; i += WAVE) {
                int p = i ^ j;
                if (p > i) {
                    int32_t a = buf[i], b = buf[p];
                    bool up = (i & k) == 0;
                    if ((a > b) == up) { buf[i] = b; buf[p] = a; }
                }
            }
            wave_sync();
        }
    }
}

// x of lane ln ^ J without an LDS round trip: DPP quad permutes (1, 2), row shifts (4), row
// rotate (8), and gfx950's permlane swaps (16, 32).  A swap of x with itself yields the two
// halves {[lo, lo], [hi, hi]} (rows for 16); whichever of them does not hold this lane's own
// value at this lane holds the partner's (and if both do, the two values are equal).
template <int J>
__device__ __forceinline__ int32_t lane_xor(int32_t x) {
    if constexpr (J == 1) {
        return __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
    } else if constexpr (J == 2) {
        return __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
    } else if constexpr (J == 4) {
        const int32_t up = __builtin_amdgcn_update_dpp(0, x, 0x104, 0xf, 0xf, false);   // row_shl:4 (lane + 4)
        const int32_t dn = __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);   // row_shr:4 (lane - 4)
        return (lane_id() & 4) ? dn : up;
    } else if constexpr (J == 8) {
        return __builtin_amdgcn_update_dpp(0, x, 0x128, 0xf, 0xf, false);   // row_ror:8
    } else if constexpr (J == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap((uint32_t)x, (uint32_t)x, false, false);
        return (int32_t)((int32_t)r[0] == x ? r[1] : r[0]);
    } else {
        static_assert(J == 32, "lane_xor: J in {1, 2, 4, 8, 16, 32}");
        const auto r = __builtin_amdgcn_permlane32_swap((uint32_t)x, (uint32_t)x, false, false);
        return (int32_t)((int32_t)r[0] == x ? r[1] : r[0]);
    }
}
__device__ __forceinline__ int32_t lane_xor(int32_t x, int j) {   // j a compile-time constant after unrolling
    switch (j) {
        case 1: return lane_xor<1>(x);
        case 2: return lane_xor<2>(x);
        case 4: return lane_xor<4>(x);
        case 8: return lane_xor<8>(x);
        case 16: return lane_xor<16>(x);
        default: return lane_xor<32>(x);
    }
}

// Bitonic sort of buf[0..n), n <= 64*E, in registers: element i = k*64 + lane lives in x[k];
// exchanges at distance >= 64 stay inside a lane, shorter ones are lane-xor shuffles.
// Padding is INT32_MAX; one load and one store per element.
// NB < 64 (E == 1, n <= NB): the merge stages stop at block size NB; the padding above NB
// stays in place (every exchange of a stage with block size kk stays inside its block).
template <int E, int NB = E * WAVE>
__device__ __forceinline__ int32_t reg_bitonic_sort(int32_t *buf, int32_t n) {   // returns element ln
    const int ln = lane_id();
    int32_t x[E];
#pragma unroll
    for (int k = 0; k < E; k++) x[k] = k * WAVE + ln < n ? buf[k * WAVE + ln] : INT32_MAX;
#pragma unroll
    for (int kk = 2; kk <= NB; kk <<= 1) {
#pragma unroll
        for (int j = kk >> 1; j > 0; j >>= 1) {
            if (j >= WAVE) {
                const int kj = j / WAVE;
#pragma unroll
                for (int k = 0; k < E; k++) {
                    if (k & kj) continue;
                    const bool asc = ((k * WAVE + ln) & kk) == 0;
                    const int32_t a = x[k], b = x[k | kj];
                    x[k] = asc ? min(a, b) : max(a, b);
                    x[k | kj] = asc ? max(a, b) : min(a, b);
                }
            } else {
#pragma unroll
                for (int k = 0; k < E; k++) {
                    const int i = k * WAVE + ln;
                    const int32_t y = lane_xor(x[k], j);
                    x[k] = (((i & j) == 0) == ((i & kk) == 0)) ? min(x[k], y) : max(x[k], y);
                }
            }
        }
    }
    wave_sync();
#pragma unroll
    for (int k = 0; k < E; k++) buf[k * WAVE + ln] = x[k];
    return x[0];
}

__device__ __forceinline__ int32_t ref_abs(int32_t a) { return a < 0 ? -a : a; }   // refinement.h:41

__device__ __forceinline__ int32_t first_greater(const int32_t *buf, int32_t l, int32_t h, int64_t key) {
    while (l < h) {
        int32_t m = (l + h) >> 1;
        if ((int64_t)buf[m] > key) h = m; else l = m + 1;
    }
    return l;
}
__device__ __forceinline__ int32_t first_geq(const int32_t *buf, int32_t l, int32_t h, int64_t key) {
    while (l < h) {
        int32_t m = (l + h) >> 1;
        if ((int64_t)buf[m] >= key) h = m; else l = m + 1;
    }
    return l;
}

__device__ SVT_COLD int32_t mean_round(int64_t tot, int32_t cnt) {   // cold: the 64-bit division
    // (int)((uint64 total + count/2) / count), refinement.c:66
    uint64_t t = (uint64_t)tot + (uint64_t)(int64_t)(cnt / 2);
    return (int32_t)(uint32_t)(t / (uint64_t)(int64_t)cnt);
}

// mean_round of a cluster whose smallest value is `base`.  With base >= 0 every value is
// >= 0, the reference's uint64 total is the exact sum, and (sum + cnt/2) / cnt =
// base + (sum - cnt*base + cnt/2) / cnt: a 32-bit division whenever the offsets' sum fits.
__device__ __forceinline__ int32_t mean_cluster(int64_t tot, int32_t cnt, int32_t base) {
    if (base >= 0) {
        const int64_t d = tot - (int64_t)cnt * (int64_t)base;
        if (d < (int64_t)0x7fffffff) {
            const uint32_t q = ((uint32_t)d + (uint32_t)(cnt / 2)) / (uint32_t)cnt;
            return (int32_t)((uint32_t)base + q);
        }
    }
    return mean_round(tot, cnt);
}

// Band filter (exact): consensus_pos only ever reads elements within `range` of pos and
// their clusters (within ci of them), i.e. values in (pos - range - ci, pos + range + ci),
// plus three facts about the whole multiset: whether any element is <= pos+25 (where the
// left pass starts, lower_bound), its minimum (upper_bound's A[0] < pos-25 test and the
// right pass's first element) and its maximum (the right pass's start when that test
// fails).  Both passes stop at the first out-of-range element, and every element between
// the band and the pass start is out of range, so voting over the band's sorted elements
// with those three facts visits the same elements with the same clusters.  Requires
// range > 25 (the left start pos+25 is then inside the band) and |pos|, |values| < 2^30
// (the reference's int32 differences cannot wrap); otherwise the full multiset is voted.
struct Band {
    bool on = false;    // the vote runs over the band's elements (else over the full multiset)
    bool f32 = false;   // ... and every band element is >= 0: 32-bit cluster sums (vote<true>)
    int32_t u = 0;      // #elements <= pos+25 of the full multiset (the left pass start)
    int32_t n_lt = 0;   // #elements <  pos-25 (upper_bound's A[0] < pos-25 test)
    int32_t n_le = 0;   // #elements <= lo (is the full minimum inside the band?)
    int32_t n_ge = 0;   // #elements >= hi (is the full maximum inside the band?)
    int32_t lo = 0, hi = 0;   // the band: open interval (lo, hi)
};

// Compacts buf[0..n) (n <= 4*WAVE) to its band elements in place; returns their count.
// Counts only (ballots), no reductions; int32 compares throughout, since the band is only
// used when |pos| < 2^30 and range + max(ci, 0) <= 2^22 (so lo, hi fit) and every element
// is within +-2^30.
__device__ __forceinline__ int32_t band_filter(int32_t *buf, int32_t n, int32_t pos, const KParams &k, Band &bd) {
    constexpr int32_t LIM = 1 << 30, WMAX = 1 << 22;
    if (k.range <= SV_MIN_LENGTH / 2 || pos <= -LIM || pos >= LIM || k.range > WMAX || k.ci > WMAX - k.range ||
        k.ci < -WMAX)
        return n;
    const int ln = lane_id();
    const int32_t w = k.range + max(k.ci, 0);
    const int32_t lo = pos - w, hi = pos + w;
    constexpr int E = 4;
    int32_t x[E];
    int32_t u = 0, nlt = 0, nle = 0, nge = 0;
    uint64_t bad = 0, neg = 0;
#pragma unroll
    for (int q = 0; q < E; q++) {
        x[q] = 0;
        if (q * WAVE >= n) break;   // wave-uniform: blocks past n hold nothing
        const int i = q * WAVE + ln;
        const bool v = i < n;
        x[q] = v ? buf[i] : 0;
        u += __popcll(ballot(v && x[q] <= pos + SV_MIN_LENGTH / 2));
        nlt += __popcll(ballot(v && x[q] < pos - SV_MIN_LENGTH / 2));
        nle += __popcll(ballot(v && x[q] <= lo));
        nge += __popcll(ballot(v && x[q] >= hi));
        bad |= ballot(v && (x[q] <= -LIM || x[q] >= LIM));
        neg |= ballot(v && lo < x[q] && x[q] < hi && x[q] < 0);
    }
    if (bad) return n;
    bd.on = true;
    bd.f32 = neg == 0;
    bd.u = u; bd.n_lt = nlt; bd.n_le = nle; bd.n_ge = nge;
    bd.lo = lo; bd.hi = hi;
    wave_sync();
    int32_t cnt = 0;
#pragma unroll
    for (int q = 0; q < E; q++) {
        if (q * WAVE >= n) break;
        const int i = q * WAVE + ln;
        const bool keep = i < n && lo < x[q] && x[q] < hi;
        const uint64_t m = ballot(keep);
        if (keep) buf[cnt + (int32_t)mbcnt(m)] = x[q];
        cnt += (int32_t)__popcll(m);
    }
    wave_sync();
    return cnt;
}

// band_filter for any n (the spill slab, > 4*WAVE candidates): the same counts and the same
// in-place compaction, 64 elements per step (writes never pass the block being read).
__device__ __forceinline__ int32_t band_filter_large(int32_t *buf, int32_t n, int32_t pos, const KParams &k,
                                                     Band &bd) {
    constexpr int32_t LIM = 1 << 30, WMAX = 1 << 22;
    if (k.range <= SV_MIN_LENGTH / 2 || pos <= -LIM || pos >= LIM || k.range > WMAX || k.ci > WMAX - k.range ||
        k.ci < -WMAX)
        return n;
    const int ln = lane_id();
    const int32_t w = k.range + max(k.ci, 0);
    const int32_t lo = pos - w, hi = pos + w;
    int32_t u = 0, nlt = 0, nle = 0, nge = 0;
    uint64_t bad = 0, neg = 0;
    for (int32_t b = 0; b < n; b += WAVE) {
        const int32_t i = b + ln;
        const bool v = i < n;
        const int32_t x = v ? buf[i] : 0;
        u += __popcll(ballot(v && x <= pos + SV_MIN_LENGTH / 2));
        nlt += __popcll(ballot(v && x < pos - SV_MIN_LENGTH / 2));
        nle += __popcll(ballot(v && x <= lo));
        nge += __popcll(ballot(v && x >= hi));
        bad |= ballot(v && (x <= -LIM || x >= LIM));
        neg |= ballot(v && lo < x && x < hi && x < 0);
    }
    if (bad) return n;
    bd.on = true;
    bd.f32 = neg == 0;
    bd.u = u; bd.n_lt = nlt; bd.n_le = nle; bd.n_ge = nge;
    bd.lo = lo; bd.hi = hi;
    wave_sync();
    int32_t cnt = 0;
    for (int32_t b = 0; b < n; b += WAVE) {
        const int32_t i = b + ln;
        const int32_t x = i < n ? buf[i] : 0;
        const bool keep = i < n && lo < x && x < hi;
        const uint64_t m = ballot(keep);
        wave_sync();
        if (keep) buf[cnt + (int32_t)mbcnt(m)] = x;
        cnt += (int32_t)__popcll(m);
        wave_sync();
    }
    return cnt;
}

__device__ __forceinline__ int32_t first_greater32(const int32_t *buf, int32_t l, int32_t h, int32_t key) {
    while (l < h) {
        int32_t m = (l + h) >> 1;
        if (buf[m] > key) h = m; else l = m + 1;
    }
    return l;
}
__device__ __forceinline__ int32_t first_geq32(const int32_t *buf, int32_t l, int32_t h, int32_t key) {
    while (l < h) {
        int32_t m = (l + h) >> 1;
        if (buf[m] >= key) h = m; else l = m + 1;
    }
    return l;
}

// consensus_pos (refinement.c:41-101) on sorted A[0..n) with prefix sums P[0..n].
// reg: x0 holds A[lane] for lanes < min(n, 64) (the register sorts), read instead of LDS.
// F32: A is a band with every element >= 0 and P holds 32-bit sums of A[j] - A0 (A0 = A[0]):
// the reference's rounded uint64 mean (sum + c/2) / c of a cluster of non-negative values is
// then A0 + (its offset sum + c/2) / c exactly, in 32 bits (offset sums < 2^31, band_filter).
template <bool F32>
__device__ __forceinline__ int32_t vote(const int32_t *A, const void *Pv, int32_t n, int32_t pos, const KParams &k,
                                        int32_t x0, bool reg, const Band &bd, int32_t A0) {
    const int64_t *P = reinterpret_cast<const int64_t *>(Pv);
    const uint32_t *P32 = reinterpret_cast<const uint32_t *>(Pv);
    const int ln = lane_id();
    const int32_t ci = k.ci, range = k.range;
    int32_t valL = -1, maxL = k.min_count - 1, distL = 0x7fffffff;
    int32_t valR = -1, maxR = k.min_count - 1, distR = 0x7fffffff;

    // lower_bound(A, n, pos+25): (#elements <= pos+25) - 1, clamped at 0  (refinement.c:3-10)
    int32_t u = 0;
    for (int32_t b = 0; b < n; b += WAVE) {
        int32_t i = b + ln;
        u += __popcll(ballot(i < n && (reg && b == 0 ? x0 : A[i]) <= pos + SV_MIN_LENGTH / 2));
    }
    int32_t p = u == 0 ? 0 : u - 1;
    if (bd.on) {   // A = the band of the full multiset (see Band): start where the full pass would
        p = bd.u == 0 ? 0 : u == 0 ? -1 : u - 1;   // u >= 1 elements <= pos+25 but none in the band:
        if (n == 0) p = -1;                         // the full pass stops at once (below the band)
    }

    // left pass: i = p, p-1, ... while |pos - A[i]| < range   (refinement.c:58-77)
    for (int32_t top = p; top >= 0; top -= WAVE) {
        int32_t i = top - ln;
        bool inr = i >= 0 && ref_abs(pos - A[i < 0 ? 0 : i]) < range;
        uint64_t stop = ballot(!inr);
        int lim = stop ? __builtin_ctzll(stop) : WAVE;   // lanes [0, lim) are in the pass
        int32_t cnt = 0, cand = 0;
        if (ln < lim) {
            int32_t a = A[i];
            if (F32) {
                const int32_t kk = first_geq32(A, 0, i, a - ci);   // contiguous j<i with a <= A[j]+ci
                cnt = i - kk + 1;
                cand = A0 + (int32_t)((P32[i + 1] - P32[kk] + (uint32_t)(cnt / 2)) / (uint32_t)cnt);
            } else {
                int32_t kk = first_geq(A, 0, i, (int64_t)a - ci);   // contiguous j<i with a <= A[j]+ci
                cnt = i - kk + 1;
                cand = mean_cluster(P[i + 1] - P[kk], cnt, A[kk]);
            }
        }
        // the greedy accept in pass order, visiting only elements whose count beats maxL
        const int32_t dd = ref_abs(pos - cand);
        for (int l = -1;;) {
            const uint64_t cm = ballot(ln < lim && ln > l && cnt > maxL);
            if (!cm) break;
            l = __builtin_ctzll(cm);
            const int32_t c = rdlane_i(cnt, l), v = rdlane_i(cand, l), d = rdlane_i(dd, l);
            if (d < ci) return v;                        // early return, refinement.c:67-68
            if (d < distL) { maxL = c; valL = v; distL = d; }
        }
        if (stop) break;
    }

    // upper_bound(A, n, pos-25): 0 if A[0] < pos-25 else n-1   (refinement.c:12-19)
    int32_t q = (n > 0 && (reg ? rdlane_i(x0, 0) : A[0]) < pos - SV_MIN_LENGTH / 2) ? 0 : n - 1;
    if (bd.on)   // the full multiset's A[0] / A[n-1]: in the band they are A's first / last element
        q = bd.n_lt > 0 ? (bd.n_le == 0 ? 0 : n) : (bd.n_ge == 0 ? n - 1 : n);
    for (int32_t bot = q; bot < n; bot += WAVE) {
        int32_t i = bot + ln;
        const int32_t ai = reg && bot == 0 ? x0 : A[i < n ? i : 0];
        bool inr = i < n && ref_abs(pos - ai) < range;
        uint64_t stop = ballot(!inr);
        int lim = stop ? __builtin_ctzll(stop) : WAVE;
        int32_t cnt = 0, cand = 0;
        if (ln < lim) {
            int32_t a = ai;
            if (F32) {
                const int32_t m = first_greater32(A, i + 1, n, a + ci);   // contiguous j>i with A[j] <= a+ci
                cnt = m - i;
                cand = A0 + (int32_t)((P32[m] - P32[i] + (uint32_t)(cnt / 2)) / (uint32_t)cnt);
            } else {
                int32_t m = first_greater(A, i + 1, n, (int64_t)a + ci);   // contiguous j>i with A[j] <= a+ci
                cnt = m - i;
                cand = mean_cluster(P[m] - P[i], cnt, a);
            }
        }
        const int32_t dd = ref_abs(pos - cand);
        for (int l = -1;;) {
            const uint64_t cm = ballot(ln < lim && ln > l && cnt > maxR);
            if (!cm) break;
            l = __builtin_ctzll(cm);
            const int32_t c = rdlane_i(cnt, l), v = rdlane_i(cand, l), d = rdlane_i(dd, l);
            if (d < ci) return v;                        // refinement.c:88-89
            if (d < distR) { maxR = c; valR = v; distR = d; }
        }
        if (stop) break;
    }
    return distL < distR ? valL : valR;   // refinement.c:100
}

// sliding_window_ins's vote (sliding_window.c:65-84) on sorted A[0..n) with prefix sums
// P[0..n]: for i = 0, slide, 2*slide, ...: support = #{j >= i : A[j] - A[i] <= ws}; the
// first i reaching the largest support >= min_count wins, its candidate is the rounded
// mean of A[i..i+support) in the reference's 32-bit int arithmetic (sum wraps mod 2^32).
__device__ __forceinline__ int32_t sw_vote(const int32_t *A, const int64_t *P, int32_t n, const KParams &k,
                                           int32_t &support_out) {
    const int ln = lane_id();
    const int32_t ws = k.sw_window, slide = k.sw_slide;
    const int32_t nstart = (n + slide - 1) / slide;
    int32_t best_sup = 0, best_i = -1;
    for (int32_t b = 0; b < nstart; b += WAVE) {
        const int32_t t = b + ln;
        int32_t sup = 0, i = 0;
        if (t < nstart) {
            i = t * slide;
            sup = first_greater(A, i, n, (int64_t)A[i] + ws) - i;         // :71-75
        }
        const bool ok = sup >= k.min_count;                                  // :76
        // wave max of qualifying supports; ties -> the smallest i (strict > in :76)
        int32_t m = wave_scan_max(ok ? sup : -1);
        m = rdlane_i(m, WAVE - 1);
        if (m > best_sup) {
            const uint64_t at = ballot(ok && sup == m);
            best_sup = m;
            best_i = rdlane_i(i, __builtin_ctzll(at));
        }
    }
    support_out = best_sup;
    if (best_i < 0) return -1;
    const uint32_t sum = (uint32_t)(uint64_t)(P[best_i + best_sup] - P[best_i]);      // :78-81, int wrap
    return (int32_t)(sum + (uint32_t)(best_sup / 2)) / best_sup;                      // :82
}

constexpr int V_CONSENSUS = 0, V_SLIDING = 1;

// Sort + prefix sums + vote over buf[0..n) with scratch for P (n+1 int64).
// LARGE: n > 4*WAVE is known (the spill slab): only the global bitonic + the int64 vote.
template <int VOTE, bool LARGE = false>
__device__ __forceinline__ int32_t sort_and_vote(int32_t *buf, int64_t *P, int32_t n, int32_t pos, const KParams &k,
                                                 int32_t &support, const Band *given = nullptr) {
    const int ln = lane_id();
    Band bd;
    if (given) bd = *given;   // buf already holds the band (band_filter_large)
    else if (!LARGE && VOTE == V_CONSENSUS && n <= 4 * WAVE) n = band_filter(buf, n, pos, k, bd);
    int32_t x0 = 0;   // sorted element ln, from the register sorts (no LDS read-back below)
    if (LARGE) {
        int N = 1;
        while (N < n) N <<= 1;
        for (int i = n + ln; i < N; i += WAVE) buf[i] = INT32_MAX;
        wave_sync();
        wave_bitonic_sort(buf, N);
    } else if (n <= 16) x0 = reg_bitonic_sort<1, 16>(buf, n);
    else if (n <= 32) x0 = reg_bitonic_sort<1, 32>(buf, n);
    else if (n <= WAVE) x0 = reg_bitonic_sort<1>(buf, n);
    else if (n <= 2 * WAVE) x0 = reg_bitonic_sort<2>(buf, n);
    else if (n <= 4 * WAVE) x0 = reg_bitonic_sort<4>(buf, n);
    else {
        int N = 1;
        while (N < n) N <<= 1;
        for (int i = n + ln; i < N; i += WAVE) buf[i] = INT32_MAX;
        wave_sync();
        wave_bitonic_sort(buf, N);
    }
    if (!LARGE && VOTE == V_CONSENSUS && bd.on && bd.f32) {   // 32-bit offset sums (see vote<true>)
        uint32_t *P32 = reinterpret_cast<uint32_t *>(P);
        const int32_t A0 = n > 0 ? rdlane_i(x0, 0) : 0;
        uint32_t carry = 0;
        if (ln == 0) P32[0] = 0;
        for (int32_t b = 0; b < n; b += WAVE) {
            const int32_t i = b + ln;
            const uint32_t x = i < n ? (uint32_t)((b == 0 ? x0 : buf[i]) - A0) : 0u;
            const uint32_t sc = carry + wave_scan_add(x);
            if (i < n) P32[i + 1] = sc;
            carry = rdlane(sc, WAVE - 1);
        }
        wave_sync();
        if (SVT_DIAG == 5) return n;
        return vote<true>(buf, P32, n, pos, k, x0, true, bd, A0);
    }
    int64_t carry = 0;
    if (ln == 0) P[0] = 0;
    for (int32_t b = 0; b < n; b += WAVE) {
        int32_t i = b + ln;
        int64_t x = i < n ? (int64_t)(!LARGE && b == 0 && n <= 4 * WAVE ? x0 : buf[i]) : 0;
        int64_t s = carry + wave_scan_add64(x);
        if (i < n) P[i + 1] = s;
        carry = (int64_t)rdlane64((uint64_t)s, WAVE - 1);
    }
    wave_sync();
    if (SVT_DIAG == 5) return n;   // diagnostic build: sort + prefix sums, no vote
    if (VOTE == V_SLIDING) return sw_vote(buf, P, n, k, support);
    return vote<false>(buf, P, n, pos, k, x0, !LARGE && n <= 4 * WAVE, bd, 0);
}

struct WinLds {
    int64_t pre[CAP + 1];         // the wave-wide vote's prefix sums
    int32_t cand[CAP];
    int32_t ncand;
};

// The window gather: the span walk (gather_span).  Round 1-2's A/B variants (per-read, CIGAR
// stream, chunk index, candidate-op lists) are retired; G stays a template parameter of the
// wave-wide window path so that diagnostic builds can plug a gather in.
constexpr int G_SPAN = 4;

template <int KIND, bool COUNT, int G>
__device__ __forceinline__ int32_t gather(const KArgs &a, int tid, uint32_t s, uint32_t e, Sink &sink, WinStats &st,
                                          WinLds &L) {
    if (lane_id() == 0) *sink.cnt = 0;
    wave_sync();
    static_assert(G == G_SPAN, "span walk only");
    (void)L;
    gather_span<KIND, COUNT>(a.pile, a.prm, tid, s, e, sink, st);
    wave_sync();
    return uniform_i(*sink.cnt);
}

template <int KIND, bool COUNT, int G, int VOTE>
__device__ __forceinline__ int32_t vote_window(const KArgs &a, WinLds &lds, int chrom, uint32_t s, uint32_t e,
                                               uint32_t imprecise, int32_t n, unsigned long long *wk, int32_t &support);

template <int KIND, bool COUNT, int G, int VOTE = V_CONSENSUS>
__device__ __forceinline__ int32_t refine_window(const KArgs &a, WinLds &lds, int chrom, uint32_t s, uint32_t e, uint32_t imprecise,
                                 unsigned long long *wk, int32_t &support) {
    WinStats st;
    Sink sink{lds.cand, CAP, &lds.ncand};
    int32_t n = gather<KIND, COUNT, G>(a, chrom - 1, s, e, sink, st, lds);
    if (COUNT && lane_id() == 0) {
        wk[W_WINDOWS] += 1; wk[W_READS] += st.reads; wk[W_OPS] += st.ops; wk[W_CANDS] += (unsigned long long)n;
        wk[W_QUERIES] += st.queries; wk[W_PROBE] += st.probe; wk[W_RANGE] += st.range; wk[W_LREADS] += st.lreads;
        wk[W_LENTRIES] += st.lentries; wk[W_STOPS] += st.stops; wk[W_STOPCH] += st.stopch;
        wk[W_SQUERIES] += st.squeries; wk[W_SPAN] += st.span;
    }
    return vote_window<KIND, COUNT, G, VOTE>(a, lds, chrom, s, e, imprecise, n, wk, support);
}

// After the gather: n candidates in lds.cand (the first CAP of them) -> consensus_pos.
template <int KIND, bool COUNT, int G, int VOTE>
__device__ __forceinline__ int32_t vote_window(const KArgs &a, WinLds &lds, int chrom, uint32_t s, uint32_t e,
                                               uint32_t imprecise, int32_t n, unsigned long long *wk, int32_t &support) {
    support = 0;
    if (n < a.prm.min_count) return -1;                    // refinement.c:43-45 (sliding: no support >= min_count)
    if (SVT_DIAG == 4) return n;   // diagnostic build: no sort/vote
    if (n <= CAP) return sort_and_vote<VOTE>(lds.cand, lds.pre, n, (int32_t)imprecise, a.prm, support);
    // spill: a slab for N ints + (n+1) int64 from the device pool, then re-gather into it
    if (COUNT && lane_id() == 0) wk[W_SPILLED] += 1;
    int N = 1;
    while (N < n) N <<= 1;
    unsigned long long words = (unsigned long long)N + 2ull * (unsigned long long)(n + 2);
    // the pool restarts for every launch: a head word tagged with another launch's epoch
    // counts as empty (no per-launch reset on the host)
    unsigned long long base = 0;
    if (lane_id() == 0) {
        unsigned long long old = __hip_atomic_load(a.pool_head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), seen;
        do {
            seen = old;
            base = (uint32_t)(seen >> 40) == a.epoch ? (seen & ((1ull << 40) - 1ull)) : 0ull;
            old = atomicCAS(a.pool_head, seen, ((unsigned long long)a.epoch << 40) | (base + words));
        } while (old != seen);
    }
    base = rdlane64(base, 0);
    if (base + words > a.pool_words) {
        if (lane_id() == 0) atomicOr(a.status, 1);
        return -1;
    }
    int32_t *g = a.pool + base;
    int64_t *gp = (int64_t *)(a.pool + ((base + (unsigned long long)N + 1ull) & ~1ull));
    WinStats st2;
    Sink s2{g, N, &lds.ncand};
    gather<KIND, false, G>(a, chrom - 1, s, e, s2, st2, lds);
    if (VOTE == V_CONSENSUS) {   // the exact band first: usually small enough for the register sort
        Band bd;
        const int32_t nb = band_filter_large(g, n, (int32_t)imprecise, a.prm, bd);
        if (bd.on && nb <= CAP) {
            for (int32_t i = lane_id(); i < nb; i += WAVE) lds.cand[i] = g[i];
            wave_sync();
            return sort_and_vote<VOTE>(lds.cand, lds.pre, nb, (int32_t)imprecise, a.prm, support, &bd);
        }
        if (bd.on) return sort_and_vote<VOTE, true>(g, gp, nb, (int32_t)imprecise, a.prm, support, &bd);
    }
    return sort_and_vote<VOTE, true>(g, gp, n, (int32_t)imprecise, a.prm, support);
}

constexpr int LV_WMAX = 1023;   // band half-width for 16-bit offsets and prefix sums (32 * 2046 < 2^16)

#include "svt_bucket.inc"

// One wave per query window, WPB independent waves per workgroup.  Window g < n is locus
// g's first window (DEL: refine_start over [pos-wider, pos+narrow], INS: refine_ins),
// window n + i is locus i's second (DEL: refine_end over end +- narrow): the wide windows
// are dispatched first, so the short ones fill the tail.
// (Workgroups in dispatch order: an XCD-aware swizzle -- each XCD a contiguous run of
// neighbouring loci -- measured slower, 37.1 vs 35.3 us on cfg2: the launch's records stay in
// the MALL across launches, so L2 locality buys nothing.)
constexpr int WPB = 4;

// The refine kernels are held to 64 VGPRs = 8 waves per SIMD (the CU's maximum): their walks
// are bound by dependent-load latency, so resident waves are what hide it.
#ifndef SVT_REFINE_WAVES
#define SVT_REFINE_WAVES 8
#endif
#define SVT_OCC __attribute__((amdgpu_waves_per_eu(SVT_REFINE_WAVES, SVT_REFINE_WAVES)))
template <bool COUNT, int G>
__device__ __forceinline__ void refine_body(const KArgs &a);

template <bool COUNT, int G>
__global__ __launch_bounds__(64 * WPB) void refine_kernel(KArgs a) { refine_body<COUNT, G>(a); }

__global__ __launch_bounds__(64 * WPB) SVT_OCC void refine_span_kernel(KArgs a) { refine_body<false, G_SPAN>(a); }

__device__ __forceinline__ void write_result(const KArgs &a, uint32_t li, uint32_t w, uint32_t r) {
    if (a.rec_out) {   // gather record {index, start, end, 0}
        uint32_t *o = reinterpret_cast<uint32_t *>(a.rec_out + li);
        o[1 + w] = r;
        if (w == 0) {
            o[0] = a.rec_index ? a.rec_index[li] : a.rec_base + li;
            o[3] = 0u;
        }
    } else {
        uint32_t *o = reinterpret_cast<uint32_t *>(a.out + li);
        o[w] = r;
    }
}

// The gather of one window kind (+ the COUNT builds' work counters); the candidates are
// left in lds.cand, their count is returned.
template <int KIND, bool COUNT, int G>
__device__ __forceinline__ int32_t gather_window(const KArgs &a, WinLds &lds, int chrom, uint32_t s, uint32_t e,
                                                 unsigned long long *wk) {
    WinStats st;
    Sink sink{lds.cand, CAP, &lds.ncand};
    const int32_t n = gather<KIND, COUNT, G>(a, chrom - 1, s, e, sink, st, lds);
    if (COUNT && lane_id() == 0) {
        wk[W_WINDOWS] += 1; wk[W_READS] += st.reads; wk[W_OPS] += st.ops; wk[W_CANDS] += (unsigned long long)n;
        wk[W_QUERIES] += st.queries; wk[W_PROBE] += st.probe; wk[W_RANGE] += st.range; wk[W_LREADS] += st.lreads;
        wk[W_LENTRIES] += st.lentries; wk[W_STOPS] += st.stops; wk[W_STOPCH] += st.stopch;
        wk[W_SQUERIES] += st.squeries; wk[W_SPAN] += st.span;
    }
    return n;
}

template <bool COUNT, int G>
__device__ __forceinline__ void refine_body(const KArgs &a) {
    __shared__ WinLds lds_all[WPB];
    const uint32_t wid = threadIdx.x >> 6;
    const uint32_t g = blockIdx.x * WPB + wid;
    if (g >= 2 * a.n) return;
    WinLds &lds = lds_all[wid];
    const uint32_t w = g >= a.n ? 1u : 0u, li = g - w * a.n;
    const svt_locus L = a.loci[li];
    const int32_t type = uniform_i(L.type), chrom = uniform_i(L.chrom);
    const uint32_t pos = (uint32_t)uniform_i((int32_t)L.pos), end = (uint32_t)uniform_i((int32_t)L.end);
    unsigned long long wk[W_N] = {};
    const KParams &k = a.prm;
    // A2 (audit.c:176-225): the window of this wave.  INV: refine_point collects only when
    // sv_type == SV_INS (refinement.c:250), so both windows vote on 0 candidates -> -1 for
    // every min_count >= 1 (validated): NA, NA.
    int kind = -1;
    uint32_t s = 0, e = 0, imp = 0;
    if (type == T_INS && w == 0) {
        kind = K_INS; s = pos - (uint32_t)k.median; e = pos + (uint32_t)k.median; imp = pos;
    } else if (type == T_DEL) {
        if (w == 0) { kind = K_START; s = pos - (uint32_t)k.wider; e = pos + (uint32_t)k.narrow; imp = pos; }
        else { kind = K_END; s = end - (uint32_t)k.narrow; e = end + (uint32_t)k.narrow; imp = end; }
    }
    uint32_t r = SVT_NA;
    // the value buckets first (svt_bucket.inc); the span lists for the windows they do not take
    const bool bk_done = !COUNT && kind >= 0 && refine_any_bk<false>(a, lds, kind, chrom, s, e, imp, wk, r);
    if (kind >= 0 && !bk_done) {
        // the kind-specific gathers, then ONE copy of the sort + vote for all kinds (code size:
        // the three inlined copies of the vote no longer compete for the instruction cache)
        int32_t n;
        if (kind == K_INS) n = gather_window<K_INS, COUNT, G>(a, lds, chrom, s, e, wk);
        else if (kind == K_START) n = gather_window<K_START, COUNT, G>(a, lds, chrom, s, e, wk);
        else n = gather_window<K_END, COUNT, G>(a, lds, chrom, s, e, wk);
        n = uniform_i(n);
        int32_t sup = 0;
        if (n < k.min_count) r = SVT_NA;                    // refinement.c:43-45
        else if (SVT_DIAG == 4) r = (uint32_t)n;           // diagnostic build: no sort/vote
        else if (n <= CAP) r = (uint32_t)sort_and_vote<V_CONSENSUS>(lds.cand, lds.pre, n, (int32_t)imp, k, sup);
        else if (kind == K_INS) r = (uint32_t)vote_window<K_INS, COUNT, G, V_CONSENSUS>(a, lds, chrom, s, e, imp, n, wk, sup);
        else if (kind == K_START) r = (uint32_t)vote_window<K_START, COUNT, G, V_CONSENSUS>(a, lds, chrom, s, e, imp, n, wk, sup);
        else r = (uint32_t)vote_window<K_END, COUNT, G, V_CONSENSUS>(a, lds, chrom, s, e, imp, n, wk, sup);
        if (COUNT) {   // what the bucket path reads for this window (its result is the same)
            wave_sync();
            uint32_t rb = 0;
            (void)refine_any_bk<true>(a, lds, kind, chrom, s, e, imp, wk, rb);
        }
    }
    if (lane_id() == 0) {
        write_result(a, li, w, r);
        if (COUNT)
            for (int i = 0; i < W_N; i++)
                if (wk[i]) atomicAdd(a.work + i, wk[i]);
    }
}

// ------------------------------------------------------------------ lane-vote kernel
// The default timed kernel.  A wave takes LV_W consecutive windows.  Phase 1, per window
// and wave-wide: the A2 window, the span query and walk (A3-A7) and the exact band filter
// (band_filter); a window whose band holds <= LV_CAP elements, all >= 0, within +-1023 of
// pos (the common case: ~20 candidates of its own breakpoint) is staged in LDS as 16-bit
// offsets from the band's low end, with the band's three whole-multiset facts.  Phase 2,
// one LANE per staged window: an in-register sorting network over the lane's offsets,
// 16-bit prefix sums, and consensus_pos (refinement.c:41-101) run per lane as the
// reference's own loops -- with the cluster starts/ends as two pointers that only move
// one way along a pass -- so the sort and the vote cost a few instructions per window
// instead of a wave-wide network and per-lane searches for every window.  Phase 3: the
// other windows (band off, > LV_CAP band elements, > CAP candidates) are re-gathered and
// voted wave-wide (refine_window), as refine_span_kernel does.  Same results.
// windows per wave (<= 64: one lane each in phase 2): 32, or 8 for batches too small to fill
// the chip with 32 per wave (svt_ctx::launch)
constexpr int LV_CAP = 32;   // band elements a lane votes on
constexpr int LV_S = 34;     // u16 per staged row (17 words: odd -> no bank conflicts)
static_assert(LV_S > LV_CAP, "a staged row needs a spare slot past LV_CAP");
// LV_BELOW / LV_ABOVE: some candidate lies at or below the band's low end / at or above its high
// end (with the band itself they give band_filter's whole-multiset facts, see lane_vote)
constexpr uint32_t LV_PENDING = 1u << 8, LV_BELOW = 1u << 9, LV_ABOVE = 1u << 10,
                   LV_REDO = 1u << 13;

struct LvMeta {
    int32_t lo;       // the band's low end (pos - w, w = range + max(ci, 0))
    uint32_t liw;     // li << 1 | w
    uint32_t flags;   // nb | LV_* bits
    int32_t n;        // candidates (min_count test)
};
constexpr uint32_t LV_NONE = 1u << 14;   // no window (INV / other types): NA
// diagnostic build 11: why a window left the lane path (bits 16+), reported as its result
#if SVT_DIAG == 11
#define LV_WHY(r) ((uint32_t)(r) << 16)
#else
#define LV_WHY(r) 0u
#endif

// Phase 1's packed walk: the windows with a span to walk, in wave order, one entry
// each (written by their phase-0 lanes); consecutive windows of <= 64 events together share
// one 64-event slot.
struct alignas(16) LvWin {
    uint64_t e0;    // the span's first event
    uint32_t s, e;  // the window
    int32_t lo;     // the band's low end
    uint32_t kl;    // kind | the window's lane (row) << 8
    uint32_t len;   // span events (> 0)
    uint32_t pad;   // value buckets: LV_BELOW when the prefix maxima below the band's buckets hold a candidate
};

template <int W>
struct LaneLds {
    uint16_t stage[W * LV_S];   // parked queries (phase 0 -> 1), band offsets (1 -> 2)
    LvMeta meta[W];
    LvWin win[W];
    uint32_t sink[WAVE];        // lane_walk: the store target of lanes without a band member
};

// Phase 1 of one window, wave-wide (A4-A7 + the band): the window's span events [E0, E0+len)
// are tested 64 * LW_U at a time (LW_U 16-B loads per lane in flight), and each candidate goes
// straight to the exact band of consensus_pos (band_filter's rule, see there): members in
// (lo, hi) are written to the window's row as 16-bit offsets from lo, and whether any candidate
// lies at or below lo / at or above hi is accumulated per lane (with the band they give the
// whole-multiset facts, lane_vote).  Values are walk positions < 2^29 + 1 (reads reaching 2^28
// bases or position 2^29 are slow and carry no events), so every candidate is >= 0 and within
// +-2^30: no int64 path is ever needed.  refine_end's leading-S reads whose walk passes e count
// as one candidate at or above the band's high end (KParams::sent_ok).
struct LaneBand {
    int32_t nb;       // band members (> LV_CAP: the row overflowed)
    uint32_t flags;   // LV_BELOW | LV_ABOVE
};

constexpr int LW_U = 4;   // 64-event slots per step of lane_walk (loads in flight per lane)
// lane_walk reads the span through a buffer descriptor of the window's own span (wave-uniform
// base and byte count): a lane's byte offset is the constant ln * 16 (+ the slot's immediate
// offset), so a load costs no VALU address arithmetic, and a load past the span returns zeros --
// an op-0 (M) event, never a candidate -- so no clamp and no partial-slot mask either.  Spans of
// 2^27 events or more take the wave-wide path (LvQuery), so the byte count fits 32 bits.
constexpr uint32_t LW_BUF_MAX = 1u << 27;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// The min_count test (refinement.c:43) is made on the band size instead of the candidate count.
// Exact: an accepted cluster lies inside the band (its elements are within ci of an element
// within range of pos), so the vote returns -1 whenever the band holds fewer than min_count
// elements, and n < min_count implies nb < min_count.  The walk then keeps no count.

// One slot as vector arithmetic.  The kernel is bound by scalar issue (one SALU instruction per
// CU and cycle): every test is the sign bit of a difference ("fail" bits), OR-ed per lane; the
// band is one unsigned compare whose lane mask is the only ballot, and below / above accumulate
// as sign bits in VGPRs (one ballot each per window).  Exact: the operands' ranges keep every
// difference inside int32 -- walk positions and candidate values <= 2^30 + 2^28 + 1 (IX_SAT, one
// op < 2^28), endpos in [1, 2^30) (slow reads carry no events), e < 2^30 (WEXACT),
// lo >= -2^29 (lane_query), the window start clamped (LwWin).
struct LwWin {
    int32_t b1;     // max(s - 1, -2^30) + 1: the overlap test endpos > s - 1 is endpos - b1 >= 0
    uint32_t e;
    int32_t sc;     // s, or 2^31 - 1 when s >= 2^31 (a window start that wrapped: x >= s never holds)
    int32_t lo1;    // lo + 1: a value v is at or below the band when v - lo1 < 0
    int32_t hm1;    // hi - 1: at or above it when hm1 - v < 0
    uint32_t wb;    // hi - lo - 1: in the band when (uint32)(v - lo1) < wb
    int32_t em2;    // e - 2 (value buckets: the event's read is yielded when its pos <= e - 2)
};
__device__ __forceinline__ uint32_t sgn(int32_t d) { return (uint32_t)d >> 31; }
__device__ __forceinline__ uint32_t opbit(uint32_t set, uint32_t op) { return __builtin_amdgcn_ubfe(set, op, 1); }

// One 64-event slot: the band's lane mask; below / above accumulated into the sign bits of
// belv / abv; iv = the lane's candidate value.
template <int KIND, bool BK>
__device__ __forceinline__ uint64_t slot_vl(const uint4 &v, const LwWin &W, uint32_t &belv, uint32_t &abv, int32_t &iv) {
    const uint32_t op = v.y & 0xfu;
    // value buckets: the event's read must also be yielded (its pos -- v.w, v.x for a leading S --
    // below the query end); a span holds only yielded reads' events
    const uint32_t yld = BK ? sgn(W.em2 - (int32_t)v.w) : 0u;
    const uint32_t far = sgn((int32_t)v.z - W.b1) | sgn((int32_t)W.e - (int32_t)v.x) | yld;   // no overlap / not reached
    uint32_t fail;
    if (BK && KIND == K_END) {                                            // :188, :210-220
        const uint32_t isD = opbit(1u << OP_DEL, op), isL = opbit(1u << SP_LEAD, op);
        const uint32_t lead = isL & (sgn((int32_t)v.z - W.b1) ^ 1u) & (sgn((int32_t)v.x - W.sc) ^ 1u) &
                              (sgn(W.em2 - (int32_t)v.x) ^ 1u);
        const uint32_t brk = lead & sgn((int32_t)W.e - (int32_t)v.w);   // walk passes e: a value >= e + 2
        abv |= brk << 31;
        fail = ((isD & (far ^ 1u)) | (lead & (brk ^ 1u))) ^ 1u;
        iv = (int32_t)(isD ? v.x + (v.y >> 4) + 1u : v.w + 1u);
    } else if (KIND == K_INS) {                                           // refinement.c:299
        fail = far | (opbit(1u << OP_INS, op) ^ 1u);
        iv = (int32_t)v.x;
    } else if (KIND == K_START) {                                         // :124, :147
        fail = far | (opbit(1u << OP_DEL | 1u << SP_TRAIL, op) ^ 1u) |
               (opbit(1u << SP_TRAIL, op) & sgn((int32_t)v.x - W.sc));
        iv = (int32_t)v.x;
    } else {                                                              // :188, :210-220
        const uint32_t isD = opbit(1u << OP_DEL, op);
        const uint32_t lead = opbit(1u << SP_LEAD, op) & (far ^ 1u) & (sgn((int32_t)v.x - W.sc) ^ 1u);
        const uint32_t brk = lead & sgn((int32_t)W.e - (int32_t)v.w);   // walk passes e: a value >= e + 2
        abv |= brk << 31;
        fail = ((isD & (far ^ 1u)) | (lead & (brk ^ 1u))) ^ 1u;
        iv = (int32_t)(isD ? v.x + (v.y >> 4) + 1u : v.w + 1u);
    }
    const uint32_t d = (uint32_t)(iv - W.lo1);
    const uint32_t pass = (fail ^ 1u) << 31;
    belv |= d & pass;
    abv |= (uint32_t)(W.hm1 - iv) & pass;
    return ballot((d | fail << 31) < W.wb);
}

// The window's scalar inputs (base address of its span, span length, LwWin, lo, its staging
// row) come from the caller's v_readlane of per-lane values computed once per wave.  Every lane
// stores in every slot -- members to their row slot, the others to their own sink word -- so a
// slot costs no exec-mask round trip on the scalar unit.
template <int KIND, bool BK>
__device__ __forceinline__ LaneBand lane_walk(uint64_t evaddr, uint32_t len, const LwWin &W, int32_t lo, uint16_t *row,
                                              uint16_t *sink) {
    const int ln = lane_id();
    int32_t nb = 0;
    uint32_t belv = 0, abv = 0;
    for (uint32_t b = 0; b < len; b += LW_U * WAVE) {
        const uint32_t left = len - b;
        uint4 v[LW_U];
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            reinterpret_cast<void *>(evaddr + (uint64_t)b * 16u), (short)0, (int)(left * 16u), 0x00020000);
#pragma unroll
        for (int u = 0; u < LW_U; u++) {   // all four in flight at once; past the span: zeros
            const u32x4 r = __builtin_amdgcn_raw_buffer_load_b128(rs, ln * 16 + u * WAVE * 16, 0, 0);
            v[u] = make_uint4(r.x, r.y, r.z, r.w);
        }
#pragma unroll
        for (int u = 0; u < LW_U; u++) {
            if ((uint32_t)(u * WAVE) >= left) break;
            int32_t iv;
            const uint64_t mb = slot_vl<KIND, BK>(v[u], W, belv, abv, iv);
            // members past LV_CAP all land in the row's spare slot LV_CAP (the window is redone);
            // the slot is computed by every lane (the empty asm keeps the compiler from moving it
            // under a branch on the member mask), then one select
            uint32_t at = (uint32_t)min(nb + (int32_t)mbcnt(mb), LV_CAP);
            asm volatile("" : "+v"(at));
            uint16_t *dst = __builtin_amdgcn_inverse_ballot_w64(mb) ? row + at : sink;
            *dst = (uint16_t)(iv - lo);
            nb += (int32_t)__popcll(mb);
        }
    }
    const uint64_t below = ballot((int32_t)belv < 0), above = ballot((int32_t)abv < 0);
    return LaneBand{nb, (below ? LV_BELOW : 0u) | (above ? LV_ABOVE : 0u)};
}

// Two windows of the same kind with 65-128 span events each, walked together: their four slots'
// loads are in flight at once, so the pair costs one memory round trip instead of two (phase 1
// is a chain of one round trip per window per wave, ~24 a wave on cfg4).
struct LwOne {
    uint64_t base;
    uint32_t len;
    LwWin W;
    int32_t lo;
    uint16_t *row;
};
template <int KIND, bool BK>
__device__ __forceinline__ void lane_walk2(const LwOne &A, const LwOne &B, uint16_t *sink, LaneBand &ra, LaneBand &rb) {
    const int ln = lane_id();
    const __amdgpu_buffer_rsrc_t sa = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(A.base), (short)0,
                                                                        (int)(A.len * 16u), 0x00020000);
    const __amdgpu_buffer_rsrc_t sb = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(B.base), (short)0,
                                                                        (int)(B.len * 16u), 0x00020000);
    uint4 v[4];
    {
        const u32x4 r0 = __builtin_amdgcn_raw_buffer_load_b128(sa, ln * 16, 0, 0);
        const u32x4 r1 = __builtin_amdgcn_raw_buffer_load_b128(sa, ln * 16 + WAVE * 16, 0, 0);
        const u32x4 r2 = __builtin_amdgcn_raw_buffer_load_b128(sb, ln * 16, 0, 0);
        const u32x4 r3 = __builtin_amdgcn_raw_buffer_load_b128(sb, ln * 16 + WAVE * 16, 0, 0);
        v[0] = make_uint4(r0.x, r0.y, r0.z, r0.w);
        v[1] = make_uint4(r1.x, r1.y, r1.z, r1.w);
        v[2] = make_uint4(r2.x, r2.y, r2.z, r2.w);
        v[3] = make_uint4(r3.x, r3.y, r3.z, r3.w);
    }
#pragma unroll
    for (int w = 0; w < 2; w++) {
        const LwOne &O = w ? B : A;
        int32_t nb = 0;
        uint32_t belv = 0, abv = 0;
#pragma unroll
        for (int u = 0; u < 2; u++) {
            int32_t iv;
            const uint64_t mb = slot_vl<KIND, BK>(v[2 * w + u], O.W, belv, abv, iv);
            uint32_t at = (uint32_t)min(nb + (int32_t)mbcnt(mb), LV_CAP);
            asm volatile("" : "+v"(at));
            uint16_t *dst = __builtin_amdgcn_inverse_ballot_w64(mb) ? O.row + at : sink;
            *dst = (uint16_t)(iv - O.lo);
            nb += (int32_t)__popcll(mb);
        }
        const uint64_t below = ballot((int32_t)belv < 0), above = ballot((int32_t)abv < 0);
        (w ? rb : ra) = LaneBand{nb, (below ? LV_BELOW : 0u) | (above ? LV_ABOVE : 0u)};
    }
}

// One 64-event slot holding the whole spans of consecutive walkable windows win[c0..]: bit i of
// M marks the first lane of a window (bit 0 always), tot <= 64 events in all.  Lane j walks
// event j - f of the window that starts at f = the highest mark <= j, with that window's own
// s / e / band (the tests of span_cand_mask, per lane); members go to the window's row at
// their rank among its members, and each window's first lane writes its meta row (band size,
// candidates, below / above) -- everything lane_walk gives a window, for 1-64 events at once.
// The event lane ln tests in the packed slot of windows win[c0..] with marks M (value buckets: one
// event array) -- loaded ahead of the slot's tests so that a run of packed slots keeps the next
// slot's loads in flight while the current one is tested.
__device__ __forceinline__ uint4 lane_packed_load(const BkIndex &B, const LvWin *win, uint32_t c0, uint64_t M) {
    const int ln = lane_id();
    const uint64_t upto = M & ((2ull << ln) - 1ull);
    const uint32_t r = (uint32_t)__popcll(upto) - 1u, f = 63u - (uint32_t)__clzll(upto);
    const LvWin &w = win[c0 + r];
    return B.ev[w.e0 + min((uint32_t)ln - f, w.len - 1u)];
}

template <bool BK>
__device__ __forceinline__ void lane_packed(const DevPileup &P, const BkIndex &B, const LvWin *win, LvMeta *meta,
                                            uint16_t *stage, uint32_t c0, uint64_t M, uint32_t tot, int32_t bw2,
                                            const uint4 *vpre = nullptr) {
    const int ln = lane_id();
    const uint64_t upto = M & ((2ull << ln) - 1ull);   // marks at or below this lane (ln 63: all)
    const uint32_t r = (uint32_t)__popcll(upto) - 1u, f = 63u - (uint32_t)__clzll(upto);
    const LvWin w = win[c0 + r];
    const uint32_t kind = w.kl & 0xffu, k = w.kl >> 8;
    const uint4 *evb = (BK ? B.ev : kind == (uint32_t)K_INS ? P.spI : P.spD) + w.e0;
    const uint4 v = vpre ? *vpre : evb[min((uint32_t)ln - f, w.len - 1u)];   // lanes past tot: their window's last event
    const uint32_t s = w.s, e = w.e, x = v.x, op = v.y & 0xfu;
    const int32_t lo = w.lo;
    const uint64_t isI = ballot(kind == (uint32_t)K_INS), isE = ballot(kind == (uint32_t)K_END);
    const uint64_t oD = ballot(op == OP_DEL), sx = ballot(s <= x), oL = ballot(op == SP_LEAD);
    const uint64_t ovl = ballot((int32_t)v.z > (int32_t)(s - 1u));
    // value buckets: the event's read is yielded (pos < e - 1: v.w, or v.x for a leading S)
    const uint64_t yw = BK ? ballot(v.w + 2u <= e) : ~0ull, yx = BK ? ballot(x + 2u <= e) : ~0ull;
    const uint64_t base = ballot((uint32_t)ln < tot) & ovl & ballot(x <= e) & (yw | (isE & oL));
    const uint64_t lead = ballot((uint32_t)ln < tot) & ovl & isE & oL & sx & (BK ? yx : ballot(x <= e));   // :210-220
    const uint64_t brk = lead & ballot(v.w > e);
    const uint64_t cm = (base & ((isI & ballot(op == OP_INS)) | (~(isI | isE) & (oD | (ballot(op == SP_TRAIL) & sx))) |
                                 (isE & oD))) |
                        (lead & ~brk);
    const int32_t iv = (int32_t)(kind == (uint32_t)K_END ? (op == OP_DEL ? x + (v.y >> 4) + 1u : v.w + 1u) : x);
    const uint64_t gt = ballot(iv > lo), lt = ballot(iv < lo + bw2);
    const uint64_t mb = cm & gt & lt;
    if ((mb >> ln) & 1ull) {
        const uint32_t rank = mbcnt(mb) - (uint32_t)__popcll(mb & ((1ull << f) - 1ull));
        stage[k * LV_S + min(rank, (uint32_t)LV_CAP)] = (uint16_t)(iv - lo);
    }
    if ((M >> ln) & 1ull) {   // the window's first lane: its totals over lanes [ln, ln + len)
        const uint64_t rm = (w.len >= 64u ? ~0ull : ((1ull << w.len) - 1ull)) << ln;
        const uint32_t nb = (uint32_t)__popcll(mb & rm);
        const bool below = (cm & ~gt & rm) != 0ull, above = ((brk | (cm & ~lt)) & rm) != 0ull;
        meta[k].flags = nb > (uint32_t)LV_CAP ? (LV_REDO | LV_WHY(3))
                                              : nb | LV_PENDING | (below ? LV_BELOW : 0u) | (above ? LV_ABOVE : 0u) | w.pad;
        meta[k].n = 0;
    }
}

// Phase 0 fills every window's band slots with 0xffff, so phase 2 takes its band straight from
// the row (no per-slot test against the band size).  The band is sorted by Batcher's odd-even
// merge sort (19 / 63 / 191 compare-exchanges for 8 / 16 / 32 elements against 24 / 80 / 240 for
// the bitonic network, all ascending).
__device__ __forceinline__ void lv_cx(uint32_t (&x)[LV_CAP], int i, int j) {
    const uint32_t p = x[i], q = x[j];
    x[i] = min(p, q);
    x[j] = max(p, q);
}
template <int LO, int N, int R>
__device__ __forceinline__ void lv_oe_merge(uint32_t (&x)[LV_CAP]) {
    if constexpr (2 * R < N) {
        lv_oe_merge<LO, N, 2 * R>(x);
        lv_oe_merge<LO + R, N, 2 * R>(x);
#pragma unroll
        for (int i = LO + R; i + R < LO + N; i += 2 * R) lv_cx(x, i, i + R);
    } else {
        lv_cx(x, LO, LO + R);
    }
}
template <int LO, int N>
__device__ __forceinline__ void lv_oe_sort(uint32_t (&x)[LV_CAP]) {
    if constexpr (N > 1) {
        lv_oe_sort<LO, N / 2>(x);
        lv_oe_sort<LO + N / 2, N / 2>(x);
        lv_oe_merge<LO, N, 1>(x);
    }
}

// floor(x / c) for x < 2^17, 1 <= c <= 64: ((x + 1/2) * rcp(c)) lies at least 1/(2c) >= 2^-7
// inside [q, q+1) exactly, and the f32 product is within 2^-9 of it (x + 1/2 < 2^17,
// v_rcp_f32 within 1 ulp), so the truncation is exact.
__device__ __forceinline__ uint32_t div_small(uint32_t x, uint32_t c) {
    return (uint32_t)(((float)x + 0.5f) * __builtin_amdgcn_rcpf((float)c));
}

// consensus_pos (refinement.c:41-101) for one lane's staged window: B[0..nb) its band's
// sorted offsets (value - lo), w = pos - lo.  Every band value is >= 0, so the reference's
// rounded uint64 mean of a cluster is lo + (offset sum + c/2) / c.  The clusters are sliding
// windows whose ends only move one way along each pass, so their sums are kept up to date
// element by element (no prefix array).
__device__ __forceinline__ int32_t lane_vote(const uint16_t *B, int32_t nb, int32_t w, int32_t lo, uint32_t fl,
                                             const KParams &k, int32_t l0 = -1) {
    const int32_t ci = k.ci, range = k.range;
    int32_t valL = -1, maxL = k.min_count - 1, distL = 0x7fffffff;
    int32_t valR = -1, maxR = k.min_count - 1, distR = 0x7fffffff;
    // lower_bound(pos+25) over the band (refinement.c:3-10), started where the full pass would
    // (l0 >= 0: the caller counted the band elements <= pos+25 already)
    if (l0 < 0) {
        int32_t h0 = nb;
        l0 = 0;
        while (l0 < h0) {
            const int32_t md = (l0 + h0) >> 1;
            if ((int32_t)B[md] > w + SV_MIN_LENGTH / 2) h0 = md; else l0 = md + 1;
        }
    }
    // band_filter's whole-multiset facts: the band's own elements (B[0] its minimum) plus
    // whether candidates lie below / above it
    const bool below = fl & LV_BELOW, above = fl & LV_ABOVE;
    const bool u0 = !below && l0 == 0;                                          // none <= pos+25
    const bool lt = below || (nb > 0 && (int32_t)B[0] < w - SV_MIN_LENGTH / 2);   // some < pos-25
    int32_t p = u0 ? 0 : l0 == 0 ? -1 : l0 - 1;
    if (nb == 0) p = -1;
    int32_t kk = p + 1, prev = 0;   // cluster [kk, i] below i, its offset sum S
    uint32_t S = 0;
    for (int32_t i = p; i >= 0; i--) {                                       // refinement.c:58
        const int32_t a = B[i];
        if (ref_abs(w - a) >= range) break;
        if (i < p) S -= (uint32_t)prev;                                      // element i+1 leaves
        if (kk > i) { kk = i; S = (uint32_t)a; }
        while (kk > 0 && (int32_t)B[kk - 1] >= a - ci) { kk--; S += B[kk]; }   // :61-64
        prev = a;
        const int32_t c = i - kk + 1;
        if (c > maxL) {                                                      // :67-76
            const int32_t co = (int32_t)div_small(S + (uint32_t)(c / 2), (uint32_t)c);   // :65
            const int32_t d = ref_abs(w - co);
            if (d < ci) return lo + co;
            if (d < distL) { maxL = c; valL = lo + co; distL = d; }
        }
    }
    // upper_bound(pos-25) (refinement.c:12-19): the full multiset's A[0] / A[n-1]
    const int32_t q = lt ? (!below ? 0 : nb) : (!above ? nb - 1 : nb);
    int32_t m = q;   // cluster [i, m) above i
    S = 0;
    for (int32_t i = q; i < nb; i++) {                                       // :80
        const int32_t a = B[i];
        if (ref_abs(w - a) >= range) break;
        if (i > q) S -= (uint32_t)prev;                                      // element i-1 leaves
        if (m <= i) { m = i + 1; S = (uint32_t)a; }
        while (m < nb && (int32_t)B[m] <= a + ci) { S += B[m]; m++; }        // :83-86
        prev = a;
        const int32_t c = m - i;
        if (c > maxR) {                                                      // :88-97
            const int32_t co = (int32_t)div_small(S + (uint32_t)(c / 2), (uint32_t)c);   // :87
            const int32_t d = ref_abs(w - co);
            if (d < ci) return lo + co;
            if (d < distR) { maxR = c; valR = lo + co; distR = d; }
        }
    }
    return distL < distR ? valL : valR;                                      // :100
}

// One of lane_vote's two passes (right: the pass above pos - 25, refinement.c:78-98; else the
// pass below pos + 25, :56-76), written once for both directions so that the two passes of a
// window run in two lanes of one wave at once: i walks from the pass's start in direction dir,
// and the cluster's far end f moves the same way while its next element lies within ci of
// B[i].  Returns whether the pass returned early (val = that value); otherwise val / dist are
// the pass's best (-1 / INT_MAX: none).
__device__ __forceinline__ bool lane_vote_half(const uint16_t *B, int32_t nb, int32_t w, int32_t lo, uint32_t fl,
                                               const KParams &k, int32_t l0, bool right, int32_t &val, int32_t &dist) {
    const int32_t ci = k.ci, range = k.range;
    const bool below = fl & LV_BELOW, above = fl & LV_ABOVE;
    int32_t start;
    if (!right) {
        const bool u0 = !below && l0 == 0;
        start = nb == 0 ? -1 : u0 ? 0 : l0 == 0 ? -1 : l0 - 1;
    } else {
        const bool lt = below || (nb > 0 && (int32_t)B[0] < w - SV_MIN_LENGTH / 2);
        start = lt ? (!below ? 0 : nb) : (!above ? nb - 1 : nb);
    }
    const int32_t dir = right ? 1 : -1;
    int32_t mx = k.min_count - 1, f = start - dir, prev = 0;
    uint32_t S = 0;
    val = -1;
    dist = 0x7fffffff;
    for (int32_t i = start; i >= 0 && i < nb; i += dir) {
        const int32_t a = B[i];
        if (ref_abs(w - a) >= range) break;
        if (i != start) S -= (uint32_t)prev;                     // the element behind i leaves
        if ((f - i) * dir < 0) { f = i; S = (uint32_t)a; }
        for (;;) {                                               // :61-64 / :83-86
            const int32_t g = f + dir;
            if (g < 0 || g >= nb) break;
            const int32_t b = B[g];
            if ((b - a) * dir > ci) break;
            f = g;
            S += (uint32_t)b;
        }
        prev = a;
        const int32_t c = (f - i) * dir + 1;
        if (c > mx) {                                            // :67-76 / :88-97
            const int32_t co = (int32_t)div_small(S + (uint32_t)(c / 2), (uint32_t)c);
            const int32_t d = ref_abs(w - co);
            if (d < ci) { val = lo + co; return true; }
            if (d < dist) { mx = c; val = lo + co; dist = d; }
        }
    }
    return false;
}

// A2 (audit.c:176-225) for window g: kind (-1: none -> NA), s, e, pos of the vote.
__device__ __forceinline__ int window_of(const KArgs &a, uint32_t g, uint32_t &li, uint32_t &w, int32_t &chrom,
                                         uint32_t &s, uint32_t &e, uint32_t &imp) {
    w = g >= a.n ? 1u : 0u;
    li = g - w * a.n;
    const svt_locus L = a.loci[li];
    const int32_t type = uniform_i(L.type);
    chrom = uniform_i(L.chrom);
    const uint32_t pos = (uint32_t)uniform_i((int32_t)L.pos), end = (uint32_t)uniform_i((int32_t)L.end);
    const KParams &k = a.prm;
    // INV: refine_point collects only when sv_type == SV_INS (refinement.c:250): NA, NA
    if (type == T_INS && w == 0) { s = pos - (uint32_t)k.median; e = pos + (uint32_t)k.median; imp = pos; return K_INS; }
    if (type == T_DEL) {
        if (w == 0) { s = pos - (uint32_t)k.wider; e = pos + (uint32_t)k.narrow; imp = pos; return K_START; }
        s = end - (uint32_t)k.narrow; e = end + (uint32_t)k.narrow; imp = end;
        return K_END;
    }
    return -1;
}


// One window's A2 + A3 answer, computed by one lane (phase 0).  u32 words only (the rows
// it is parked in are 4-byte aligned).
constexpr int32_t LQ_REDO = 1 << 4;   // kind bit: the window takes the wave-wide path
struct LvQuery {
    int32_t kind;          // K_* (| LQ_REDO), -1: no window (NA)
    int32_t lo;            // the vote's band low end: pos - (range + max(ci, 0))
    uint32_t s, e, liw, len;        // the window, li << 1 | w, its span's event count
    uint32_t e0[2];                 // the span's first event
    uint32_t fl;                    // value buckets: LV_BELOW from the prefix maxima
};
static_assert(sizeof(LvQuery) <= LV_S * 2, "LvQuery must fit a staging row");

__device__ __forceinline__ void lane_query(const KArgs &a, uint32_t g, bool band_ok, LvQuery &q) {
    const DevPileup &P = a.pile;
    const KParams &k = a.prm;
    const uint32_t w = g >= a.n ? 1u : 0u, li = g - w * a.n;
    const svt_locus L = a.loci[li];
    q.kind = -1;
    q.liw = li << 1 | w;
    const uint32_t pos = L.pos, end = L.end;
    uint32_t imp = 0;
    if (L.type == T_INS && w == 0) { q.kind = K_INS; q.s = pos - (uint32_t)k.median; q.e = pos + (uint32_t)k.median; imp = pos; }
    else if (L.type == T_DEL && w == 0) { q.kind = K_START; q.s = pos - (uint32_t)k.wider; q.e = pos + (uint32_t)k.narrow; imp = pos; }
    else if (L.type == T_DEL) { q.kind = K_END; q.s = end - (uint32_t)k.narrow; q.e = end + (uint32_t)k.narrow; imp = end; }
    // INV: refine_point collects only when sv_type == SV_INS (refinement.c:250): NA, NA
    if (q.kind < 0) return;
    // the wave-wide path (refine_redo_kernel) when the window ends at or past WEXACT or is a
    // refine_end window whose stops need the per-read replay (gather_span), when the band is off
    // (band_ok) or pos is beyond +-2^30 (int32 differences could wrap)
    constexpr int32_t LIM = 1 << 30;
    if (q.e >= WEXACT || (q.kind == K_END && !k.sent_ok) || !band_ok || (int32_t)imp <= -LIM || (int32_t)imp >= LIM) {
        q.kind |= LQ_REDO;
        return;
    }
    q.lo = (int32_t)imp - (k.range + max(k.ci, 0));
    if (q.lo < -(1 << 29)) { q.kind |= LQ_REDO; return; }   // (keeps slot_vl's differences in int32)
    q.len = 0;   // empty span: no reads
    const int tid = L.chrom - 1;
    const int64_t beg = (int64_t)(uint32_t)(q.s - 1u), qend = (int64_t)(uint32_t)(q.e - 1u);
    if (tid < 0 || tid >= P.n_targets || qend <= beg) return;   // A3: no reads
    const int64_t ra = P.tid_off[tid], nr = P.tid_off[tid + 1] - ra;
    if (nr == 0) return;
    const int64_t b0 = P.bkt_off[tid], nb = P.bkt_off[tid + 1] - b0;   // last bucket = {nr, nr}
    const int64_t bh = min(qend >> BKT_SHIFT, nb - 1), bl = min(beg >> BKT_SHIFT, nb - 1);
    const uint2 h0 = P.bkt[b0 + bh], h1 = P.bkt[b0 + min(bh + 1, nb - 1)];
    const uint2 l0 = P.bkt[b0 + bl], l1 = P.bkt[b0 + min(bl + 1, nb - 1)];
    // hi = first read with pos >= qend in [h0.x, h1.x]; lo = first with emax > beg in [l0.y, l1.y]
    int64_t hl = h0.x, hh = h1.x, ll = l0.y, lh = l1.y;
    const int32_t *pp = P.pos + ra, *em = P.emax + ra;
    while (hl < hh || ll < lh) {   // the two binary searches interleaved (their loads overlap)
        const int64_t hm = (hl + hh) >> 1, lm = (ll + lh) >> 1;
        const int32_t pv = hl < hh ? pp[hm] : 0, evv = ll < lh ? em[lm] : 0;
        if (hl < hh) { if ((int64_t)pv >= qend) hh = hm; else hl = hm + 1; }
        if (ll < lh) { if ((int64_t)evv > beg) lh = lm; else ll = lm + 1; }
    }
    const int64_t lo = ra + ll, hi = ra + hl;
    if (lo >= hi) return;
    const uint64_t *off = q.kind == K_INS ? P.spoffI : P.spoffD;
    const uint64_t E0 = off[lo], E1 = off[hi];
    // spans of 2^27 events or more: the wave-wide path (lane_walk's buffer byte count)
    if (E1 - E0 >= (uint64_t)LW_BUF_MAX) { q.kind |= LQ_REDO; return; }
    q.e0[0] = (uint32_t)E0; q.e0[1] = (uint32_t)(E0 >> 32);
    q.len = (uint32_t)(E1 - E0);
}

// lane_query for the value buckets (svt_bucket.inc): A2, the window's eligibility, its band's bucket
// span and the prefix maxima's BELOW -- no region query, no binary search (one dependent step after
// the locus: the contig's bucket base, then the two bucket offsets and one prefix-max key).
__device__ __forceinline__ void lane_query_bk(const KArgs &a, uint32_t g, LvQuery &q) {
    const KParams &k = a.prm;
    const uint32_t w = g >= a.n ? 1u : 0u, li = g - w * a.n;
    const svt_locus L = a.loci[li];
    q.kind = -1;
    q.liw = li << 1 | w;
    q.len = 0;
    q.fl = 0;
    const uint32_t pos = L.pos, end = L.end;
    uint32_t imp = 0;
    if (L.type == T_INS && w == 0) { q.kind = K_INS; q.s = pos - (uint32_t)k.median; q.e = pos + (uint32_t)k.median; imp = pos; }
    else if (L.type == T_DEL && w == 0) { q.kind = K_START; q.s = pos - (uint32_t)k.wider; q.e = pos + (uint32_t)k.narrow; imp = pos; }
    else if (L.type == T_DEL) { q.kind = K_END; q.s = end - (uint32_t)k.narrow; q.e = end + (uint32_t)k.narrow; imp = end; }
    if (q.kind < 0) return;   // INV: refine_point collects only when sv_type == SV_INS (refinement.c:250): NA, NA
    BkWin W;
    const int el = bk_eligible(a, q.kind, L.chrom, q.s, q.e, imp, W);
    if (el == 0) { q.kind |= LQ_REDO; return; }   // the span-list path (refine_redo_kernel)
    q.lo = (int32_t)imp - (k.range + max(k.ci, 0));
    if (el < 0) return;                            // A3: no reads -> nb = 0 -> NA
    uint32_t E0, E1;
    bool below;
    bk_query(a.bk, q.kind, L.chrom - 1, W, E0, E1, below);
    if (E1 - E0 >= LW_BUF_MAX) { q.kind |= LQ_REDO; return; }   // (lane_walk's buffer byte count)
    q.e0[0] = E0;
    q.e0[1] = 0u;
    q.len = E1 - E0;
    q.fl = below ? LV_BELOW : 0u;
}

// SVT_PHASE_PROF (diagnostic builds): every wave of refine_lane_kernel adds its phases' wall
// time (100 MHz ticks) and work counts into ph_prof, read (and cleared) by svt_diag_phase.
#ifndef SVT_PHASE_PROF
#define SVT_PHASE_PROF 0
#endif
// PH(...) / PH_T(t): the instrumentation's statements, compiled out of the product.
#if SVT_PHASE_PROF
__device__ unsigned long long ph_prof[16];
#define PH_ADD(i, v) atomicAdd(&ph_prof[i], (unsigned long long)(v))
#define PH(...) __VA_ARGS__
#define PH_T(t) const long long t = wall_clock64()
#else
#define PH(...)
#define PH_T(t)
#endif
template <int LV_W, bool BK>
__global__ __launch_bounds__(64 * WPB) SVT_OCC void refine_lane_kernel(KArgs a) {
    __shared__ LaneLds<LV_W> lds_all[WPB];
    const uint32_t wid = threadIdx.x >> 6;
    const int ln = lane_id();
    const uint32_t g0 = (blockIdx.x * WPB + wid) * LV_W, nw = 2u * a.n;
    if (g0 >= nw) return;
    LaneLds<LV_W> &L = lds_all[wid];
    const KParams &k = a.prm;
    const uint32_t cnt = min((uint32_t)LV_W, nw - g0);
    const int32_t bw = k.range + max(k.ci, 0);   // the band's half-width
    PH_T(pt0);
    const bool band_ok = k.range > SV_MIN_LENGTH / 2 && bw <= LV_WMAX && k.ci >= -LV_WMAX &&
                         SVT_DIAG != 7;
    // ---- phase 0: every window's A2 + A3 at once, one lane each (the dependent loads of
    // locus -> bucket words -> pos/emax searches -> span bounds run once per LV_W windows).
    // The meta row gets its final flags here unless the window has a span to walk, and the
    // walkable windows' table entries go to win[] in lane order.
    uint32_t nwin;
    {
        const bool mine = (uint32_t)ln < cnt;
        LvQuery q{};
        if (mine) {
            if (BK) lane_query_bk(a, g0 + (uint32_t)ln, q);
            else lane_query(a, g0 + (uint32_t)ln, band_ok, q);
        }
        const bool walk = mine && q.kind >= 0 && !(q.kind & LQ_REDO) && q.len != 0u;
        if (mine) {
            uint32_t *row32 = reinterpret_cast<uint32_t *>(L.stage + (uint32_t)ln * LV_S);
#pragma unroll
            for (int j = 0; j < LV_CAP / 2; j++) row32[j] = 0xffffffffu;   // unused band slots read as 0xffff
            LvMeta m;
            m.lo = q.lo;
            m.liw = q.liw;
            m.flags = q.kind < 0 ? LV_NONE : (q.kind & LQ_REDO) ? (LV_REDO | LV_WHY(1)) : LV_PENDING;
            m.n = 0;
            L.meta[ln] = m;
        }
        const uint64_t wm = ballot(walk);
        if (walk) {
            LvWin wn;
            wn.e0 = (uint64_t)q.e0[0] | (uint64_t)q.e0[1] << 32;
            wn.s = q.s;
            wn.e = q.e;
            wn.lo = q.lo;
            wn.kl = (uint32_t)q.kind | (uint32_t)ln << 8;
            wn.len = q.len;
            wn.pad = q.fl;
            L.win[mbcnt(wm)] = wn;
        }
        nwin = (uint32_t)__popcll(wm);
    }
    wave_sync();
    PH_T(pt1);
    if (SVT_DIAG == 6) {   // diagnostic build: phase 0 only (its answers written out, so it is not dead code)
        if ((uint32_t)ln < cnt) {
            const LvMeta mt = L.meta[ln];
            const LvWin wn = L.win[min((uint32_t)ln, nwin > 0 ? nwin - 1 : 0u)];
            write_result(a, mt.liw >> 1, mt.liw & 1u, mt.flags ^ (uint32_t)wn.e0 ^ wn.len);
        }
        return;
    }
    // ---- phase 1 (packed): windows of <= 64 events share slots (lane_packed), longer ones are
    // walked alone (lane_walk).  Lane c holds walkable window c's walk constants, computed here
    // once for the wave; the scalar window loop reads them with v_readlane (no LDS round trip and
    // no scalar arithmetic per window), and a window walked alone leaves its flags in lane kw of
    // aflags (a v_cndmask on the lane index) instead of a store to its meta row.
    uint32_t aflags = 0;
    {
        const bool has = (uint32_t)ln < nwin;
        const LvWin wv = L.win[has ? (uint32_t)ln : 0u];   // (entry 0 unused when nwin == 0)
        const uint32_t lenv = has ? wv.len : 0u, klv = wv.kl, ev = wv.e, flv = wv.pad;
        const int32_t em2v = (int32_t)(wv.e - 2u);
        const int32_t lov = wv.lo;
        const int32_t b1v = max((int32_t)(wv.s - 1u), -(1 << 30)) + 1;
        const int32_t scv = (int32_t)min(wv.s, 0x7fffffffu);
        const uint64_t addrv = reinterpret_cast<uint64_t>(
            (BK ? a.bk.ev : (klv & 0xffu) == (uint32_t)K_INS ? a.pile.spI : a.pile.spD) +
            wv.e0);
        uint16_t *sink = reinterpret_cast<uint16_t *>(&L.sink[ln]);
        const int32_t bw2 = 2 * bw;
        PH({ const uint32_t tl = rdlane(wave_scan_add(lenv), WAVE - 1); if (ln == 0) { PH_ADD(8, nwin); PH_ADD(9, tl); } })
        for (uint32_t c = 0; c < nwin;) {
            const uint32_t l0 = rdlane(lenv, (int)c);
            PH(if (ln == 0) { if (l0 > (uint32_t)WAVE) { PH_ADD(10, 1); PH_ADD(11, (l0 + 255u) / 256u); } else PH_ADD(12, 1); })
            if (l0 > (uint32_t)WAVE && l0 <= 2u * WAVE && c + 1u < nwin) {   // a pair of 2-slot windows?
                const uint32_t l1 = rdlane(lenv, (int)(c + 1u));
                const uint32_t ka = rdlane(klv, (int)c), kb = rdlane(klv, (int)(c + 1u));
                if (l1 > (uint32_t)WAVE && l1 <= 2u * WAVE && ((ka ^ kb) & 0xffu) == 0u) {
                    auto one = [&](uint32_t cc, uint32_t kl, uint32_t len) {
                        const int32_t lo = rdlane_i(lov, (int)cc);
                        return LwOne{rdlane64(addrv, (int)cc), len,
                                     LwWin{rdlane_i(b1v, (int)cc), rdlane(ev, (int)cc), rdlane_i(scv, (int)cc), lo + 1,
                                           lo + bw2 - 1, (uint32_t)(bw2 - 1), rdlane_i(em2v, (int)cc)},
                                     lo, L.stage + (kl >> 8) * LV_S};
                    };
                    const LwOne A = one(c, ka, l0), B = one(c + 1u, kb, l1);
                    LaneBand ra, rb;
                    if ((ka & 0xffu) == (uint32_t)K_INS) lane_walk2<K_INS, BK>(A, B, sink, ra, rb);
                    else if ((ka & 0xffu) == (uint32_t)K_START) lane_walk2<K_START, BK>(A, B, sink, ra, rb);
                    else lane_walk2<K_END, BK>(A, B, sink, ra, rb);
                    const uint32_t fa = ra.nb > LV_CAP ? (LV_REDO | LV_WHY(3))
                                                       : (uint32_t)ra.nb | LV_PENDING | ra.flags | rdlane(flv, (int)c);
                    const uint32_t fb = rb.nb > LV_CAP ? (LV_REDO | LV_WHY(3))
                                                       : (uint32_t)rb.nb | LV_PENDING | rb.flags | rdlane(flv, (int)(c + 1u));
                    aflags = (uint32_t)ln == (ka >> 8) ? fa : (uint32_t)ln == (kb >> 8) ? fb : aflags;
                    c += 2u;
                    continue;
                }
            }
            if (l0 > (uint32_t)WAVE) {
                const uint32_t kl = rdlane(klv, (int)c), kind = kl & 0xffu, kw = kl >> 8;
                const int32_t lo = rdlane_i(lov, (int)c);
                const LwWin W{rdlane_i(b1v, (int)c), rdlane(ev, (int)c), rdlane_i(scv, (int)c), lo + 1, lo + bw2 - 1,
                              (uint32_t)(bw2 - 1), rdlane_i(em2v, (int)c)};
                const uint64_t base = rdlane64(addrv, (int)c);
                uint16_t *row = L.stage + kw * LV_S;
                LaneBand r;
                if (kind == (uint32_t)K_INS) r = lane_walk<K_INS, BK>(base, l0, W, lo, row, sink);
                else if (kind == (uint32_t)K_START) r = lane_walk<K_START, BK>(base, l0, W, lo, row, sink);
                else r = lane_walk<K_END, BK>(base, l0, W, lo, row, sink);
                const uint32_t f = r.nb > LV_CAP ? (LV_REDO | LV_WHY(3)) : (uint32_t)r.nb | LV_PENDING | r.flags | rdlane(flv, (int)c);
                aflags = (uint32_t)ln == kw ? f : aflags;
                c++;
                continue;
            }
            uint64_t M = 1ull;
            uint32_t tot = l0, c1 = c + 1u;
            for (; c1 < nwin; c1++) {
                const uint32_t l = rdlane(lenv, (int)c1);
                if (tot + l > (uint32_t)WAVE) break;
                M |= 1ull << tot;
                tot += l;
            }
            if (!BK) {
                lane_packed<BK>(a.pile, a.bk, L.win, L.meta, L.stage, c, M, tot, bw2);
                c = c1;
                continue;
            }
            // value buckets: most windows hold < 64 events, so a wave's phase 1 is a run of packed
            // slots -- each slot's events are loaded while the previous slot is tested (the loads,
            // not the tests, were the run's length: one round trip per slot, ~9 slots a wave on cfg4)
            uint4 v = lane_packed_load(a.bk, L.win, c, M);
            for (;;) {
                uint64_t Mn = 1ull;
                uint32_t totn = 0, cn1 = c1;
                const bool more = c1 < nwin && rdlane(lenv, (int)c1) <= (uint32_t)WAVE;
                if (more) {
                    totn = rdlane(lenv, (int)c1);
                    for (cn1 = c1 + 1u; cn1 < nwin; cn1++) {
                        const uint32_t l = rdlane(lenv, (int)cn1);
                        if (totn + l > (uint32_t)WAVE) break;
                        Mn |= 1ull << totn;
                        totn += l;
                    }
                }
                // (unconditional: a load under a branch would be waited for at the join)
                const uint4 vn = lane_packed_load(a.bk, L.win, more ? c1 : c, more ? Mn : M);
                lane_packed<BK>(a.pile, a.bk, L.win, L.meta, L.stage, c, M, tot, bw2, &v);
                c = c1;
                if (!more) break;
                v = vn;
                M = Mn;
                tot = totn;
                c1 = cn1;
            }
        }
        wave_sync();
    }
    PH_T(pt2);
    const bool mine = (uint32_t)ln < cnt;
    LvMeta mt = mine ? L.meta[ln] : LvMeta{0, 0, 0, 0};
    if (aflags) mt.flags = aflags;   // the window was walked alone
    if (SVT_DIAG == 8) {   // diagnostic build: phases 0-1 only (a checksum of their LDS output written out)
        if (mine) {
            const uint32_t *row32 = reinterpret_cast<const uint32_t *>(L.stage + (uint32_t)ln * LV_S);
            uint32_t h = mt.flags ^ (uint32_t)mt.lo;
            for (int j = 0; j < LV_S / 2; j++) h = h * 31u + row32[j];
            write_result(a, mt.liw >> 1, mt.liw & 1u, h);
        }
        return;
    }
    // ---- phase 2: one lane per staged window
    uint64_t redo;   // phase 3's windows (the meta rows are overwritten by its gathers)
    {
        // decisions: no window or fewer than min_count band members -> NA (refinement.c:43-45,
        // LaneBand); the wave-wide path; or this lane's vote
        const bool na = mine && ((mt.flags & LV_NONE) || (!(mt.flags & LV_REDO) && (int32_t)(mt.flags & 0xffu) < k.min_count));
        if (na) write_result(a, mt.liw >> 1, mt.liw & 1u, SVT_NA);
        redo = ballot(mine && !na && (mt.flags & LV_REDO));
        const bool pend = mine && !na && !(mt.flags & LV_REDO) && (mt.flags & LV_PENDING);
        const int32_t nb = pend ? (int32_t)(mt.flags & 0xffu) : 0;
        const uint64_t any = ballot(pend);
        if (any) {
            uint32_t x[LV_CAP];
            // lanes without a staged window use row 0 read-only (rows exist for LV_W lanes only)
            uint16_t *row = L.stage + (pend ? (uint32_t)ln : 0u) * LV_S;
            const uint32_t *row32 = reinterpret_cast<const uint32_t *>(row);
#pragma unroll
            for (int j = 0; j < LV_CAP; j += 2) {   // two offsets per 4-byte LDS read
                const uint32_t v = row32[j >> 1];
                x[j] = v & 0xffffu;   // (slots past the band hold 0xffff: phase 0)
                x[j + 1] = v >> 16;
            }
            int32_t nmax = nb;   // wave max of nb: the smallest network that sorts every lane
#pragma unroll
            for (int d = 32; d > 0; d >>= 1) nmax = max(nmax, __shfl_xor(nmax, d, WAVE));
            PH(if (ln == 0) PH_ADD(nmax <= 8 ? 13 : nmax <= 16 ? 14 : 15, 1));
            if (nmax <= 8) lv_oe_sort<0, 8>(x);
            else if (nmax <= 16) lv_oe_sort<0, 16>(x);
            else lv_oe_sort<0, 32>(x);
            uint32_t *wrow = reinterpret_cast<uint32_t *>(row);
            int32_t l0 = 0;
            if (pend) {
#pragma unroll
                for (int j = 0; j < LV_CAP; j += 2) wrow[j >> 1] = x[j] | x[j + 1] << 16;
                // the band elements <= pos + 25, counted on the sorted registers (no search)
#pragma unroll
                for (int j = 0; j < LV_CAP; j++) l0 += (int32_t)(x[j] <= (uint32_t)(bw + SV_MIN_LENGTH / 2));
                l0 = min(l0, nb);
            }
            // value buckets: ABOVE was only seen as far as the band's buckets; the vote reads it
            // only when no candidate lies below pos - 25 (lane_vote's q) -- then the wave walks for
            // it, window by window (bk_above: the bounded walks of svt_bucket.inc)
            const bool needA = BK && pend && !(mt.flags & (LV_BELOW | LV_ABOVE)) &&
                               (int32_t)x[0] >= bw - SV_MIN_LENGTH / 2;
            if (BK && SVT_DIAG != 41 && SVT_DIAG != 43) {   // (41, 43: diagnostic builds, no ABOVE walks)
                for (uint64_t na = ballot(needA); na; na &= na - 1ull) {
                    const int l = __builtin_ctzll(na);
                    uint32_t li, wi, ws = 0, we = 0, wimp = 0;
                    int32_t chrom;
                    const int kind = window_of(a, g0 + (uint32_t)l, li, wi, chrom, ws, we, wimp);
                    BkWin W;
                    bool ab = false;
                    if (bk_eligible(a, kind, chrom, ws, we, wimp, W) == 1) {
                        unsigned long long wk_ = 0;
                        if (kind == K_INS) ab = bk_above<K_INS>(a.bk, chrom - 1, W, wk_);
                        else if (kind == K_START) ab = bk_above<K_START>(a.bk, chrom - 1, W, wk_);
                        else ab = bk_above<K_END>(a.bk, chrom - 1, W, wk_);
                    }
                    if (ln == l && ab) mt.flags |= LV_ABOVE;
                }
            }
            if (SVT_DIAG == 42 || SVT_DIAG == 43) {   // diagnostic builds: no vote (42), no vote or ABOVE walks (43)
                if (pend) write_result(a, mt.liw >> 1, mt.liw & 1u, x[0] + (uint32_t)l0 + (uint32_t)needA);
            } else if (SVT_VOTE2 && LV_W <= 32) {
                // the two passes of window j in lanes j (below pos + 25) and j + 32 (above pos - 25)
                const int src = ln & 31;
                const bool right = ln >= 32;
                const bool pv = __shfl((int)pend, src, WAVE) != 0;
                const int32_t nbv = __shfl(nb, src, WAVE), lov = __shfl(mt.lo, src, WAVE), l0v = __shfl(l0, src, WAVE);
                const uint32_t flv = (uint32_t)__shfl((int)mt.flags, src, WAVE);
                int32_t val = -1, dist = 0x7fffffff;
                bool early = false;
                if (pv) early = lane_vote_half(L.stage + (uint32_t)src * LV_S, nbv, bw, lov, flv, k, l0v, right, val, dist);
                const int32_t valR = __shfl(val, src + 32, WAVE), distR = __shfl(dist, src + 32, WAVE);
                const bool earlyR = __shfl((int)early, src + 32, WAVE) != 0;
                if (pend) {   // :100 after an early return of neither pass
                    const int32_t r = early ? val : earlyR ? valR : dist < distR ? val : valR;
                    write_result(a, mt.liw >> 1, mt.liw & 1u, (uint32_t)r);
                }
            } else if (pend) {
                const int32_t r = lane_vote(row, nb, bw, mt.lo, mt.flags, k, l0);
                write_result(a, mt.liw >> 1, mt.liw & 1u, (uint32_t)r);
            }
        }
        wave_sync();
    }
    PH_T(pt3);
    // ---- the windows voted wave-wide go to refine_redo_kernel (rare: 0.6 % of cfg4's)
    if (SVT_DIAG == 11) {   // diagnostic build: each left-over window's result = 0xF0000000 | its reason
        if ((redo >> ln) & 1ull) write_result(a, mt.liw >> 1, mt.liw & 1u, 0xF0000000u | (mt.flags >> 16));
        return;
    }
    if (SVT_DIAG == 9) {   // diagnostic build: count them (status word bits 8+), nothing else
        if (ln == 0 && redo) atomicAdd(a.status, (int32_t)__popcll(redo) << 8);
        return;
    }
    if (redo) {
        uint32_t base = 0;
        if (ln == 0) base = atomicAdd(a.redo_ctr, (uint32_t)__popcll(redo));
        base = rdlane(base, 0);
        if ((redo >> ln) & 1ull) a.redo_list[base + mbcnt(redo)] = g0 + (uint32_t)ln;
    }
    PH(if (ln == 0) { const long long pt4 = wall_clock64(); PH_ADD(0, pt1 - pt0); PH_ADD(1, pt2 - pt1); PH_ADD(2, pt3 - pt2); PH_ADD(3, pt4 - pt3); PH_ADD(4, 1); })
}

// The lane kernel's left-over windows (band off, > LV_CAP band elements, > CAP candidates,
// slow reads, windows ending at or past 2^31), one wave each, re-gathered and voted
// wave-wide (refine_window); the grid strides over the list.  Also resets the counter the
// next launch will use.
__global__ __launch_bounds__(64 * WPB) SVT_OCC void refine_redo_kernel(KArgs a) {
    __shared__ WinLds lds_all[WPB];
    const uint32_t wid = threadIdx.x >> 6;
    const uint32_t gw = blockIdx.x * WPB + wid, nwv = gridDim.x * WPB;
    if (gw == 0 && lane_id() == 0) *a.redo_next = 0u;
    const uint32_t cnt = (uint32_t)uniform_i((int32_t)__hip_atomic_load(a.redo_ctr, __ATOMIC_RELAXED,
                                                                         __HIP_MEMORY_SCOPE_AGENT));
    WinLds &lds = lds_all[wid];
    for (uint32_t idx = gw; idx < cnt; idx += nwv) {
        const uint32_t g = (uint32_t)uniform_i((int32_t)a.redo_list[idx]);
        uint32_t li, w, s = 0, e = 0, imp = 0;
        int32_t chrom;
        const int kind = window_of(a, g, li, w, chrom, s, e, imp);
        unsigned long long wk[W_N];
        int32_t sup;
        uint32_t r = SVT_NA;
        if (kind >= 0 && refine_any_bk<false>(a, lds, kind, chrom, s, e, imp, wk, r)) {}   // the value buckets
        else if (kind == K_INS) r = (uint32_t)refine_window<K_INS, false, G_SPAN>(a, lds, chrom, s, e, imp, wk, sup);
        else if (kind == K_START) r = (uint32_t)refine_window<K_START, false, G_SPAN>(a, lds, chrom, s, e, imp, wk, sup);
        else if (kind == K_END) r = (uint32_t)refine_window<K_END, false, G_SPAN>(a, lds, chrom, s, e, imp, wk, sup);
        if (lane_id() == 0) write_result(a, li, w, r);
        wave_sync();
    }
}

// sliding_window_ins mode (sliding_window.c:8-97): one wave per sub-window.  A sub-window
// is refine_ins's window exactly -- the same region query (sub_start-1, sub_end-1, :27),
// the same walk (I >= 50 collects rp, advance unless I/S, break when rp > sub_end,
// :30-54) -- so it reuses the stream gather; only the vote differs (sw_vote).
template <int G>
__global__ __launch_bounds__(64 * WPB) void sw_kernel(KArgs a) {
    __shared__ WinLds lds_all[WPB];
    const uint32_t wid = threadIdx.x >> 6;
    const uint32_t g = blockIdx.x * WPB + wid;
    if (g >= a.n) return;
    const uint4 q = a.sw_sub[g];
    const int32_t chrom = uniform_i((int32_t)q.x);
    const uint32_t s = (uint32_t)uniform_i((int32_t)q.y), e = (uint32_t)uniform_i((int32_t)q.z);
    unsigned long long wk[W_N];
    int32_t sup = 0;
    const int32_t c = refine_window<K_INS, false, G, V_SLIDING>(a, lds_all[wid], chrom, s, e, 0u, wk, sup);
    if (lane_id() == 0) a.sw_out[g] = make_int2(c, sup);
}

// bestCandidateOverall per query over its sub-windows in order (sliding_window.c:86-92).
__global__ void sw_reduce_kernel(const int2 *sub, const uint64_t *off, uint32_t nq, int32_t *best) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    int32_t b = -1, m = 0;
    for (uint64_t k = off[q]; k < off[q + 1]; k++) {
        const int2 v = sub[k];
        if (v.x != -1 && v.y > m) { m = v.y; b = v.x; }
    }
    best[q] = b;
}

#include "svt_index.inc"
#include "svt_index2.inc"
#include "svt_bucket_build.inc"
#include "svt_poa.inc"
#include "svt_bam.inc"

#include "svt_inflate.inc"

}  // namespace

// ====================================================================== C ABI
struct svt_ctx {
    svt_params prm{};
    int device = 0;
    bool lane_vote = true;        // refine_lane_kernel from 64K windows up; SVTREK_GATHER=span1: refine_span_kernel always
    uint64_t ix_ranges = 32768;   // index ranges per pileup (SVTREK_IX_RANGES, A/B): ~n_ops / this ops each,
                                  // at most IX_TMAX ops (and IX_RCAP reads) a range
    int lane_w = 0;               // SVTREK_LANE_W=32 forces the lane kernel at every batch size (tests)
    uint32_t *d_redo = nullptr;   // lane-vote launches: left-over window list
    size_t redo_cap = 0;
    uint32_t lane_par = 0;        // which of the two redo counters the next lane launch uses
    char err[512] = {0};
    // pileup
    int32_t n_targets = 0;
    int64_t n_reads = 0;
    uint64_t n_ops = 0;
    int32_t *d_pos = nullptr, *d_emax = nullptr;
    uint4 *d_rec = nullptr;
    uint8_t *d_clip8 = nullptr;       // per read its clip bits (rec.z >> 30) alone: the census's 1 B instead of 16
    uint64_t *d_off64 = nullptr;      // stream offsets [n_reads + 1]
    int64_t *d_tid_off = nullptr, *d_bkt_off = nullptr;
    uint2 *d_bkt = nullptr;
    uint32_t *d_cigar = nullptr;      // CIGAR stream
    uint64_t n_ins = 0;               // I >= 50 ops in the pileup (= I-list events; d_spoffI indexes them per read)
    // device index (svt_index.inc)
    uint64_t *d_part = nullptr;       // [n_ranges + 1]
    uint32_t n_ranges = 0;
    IxTot *d_agg = nullptr;           // range (group) totals
    IxTot *d_bsum = nullptr, *d_bpre = nullptr;   // their sums per block of IX_BLK, the blocks' exclusive scan
    size_t n_bsum = 0;
    bool bsum_dirty = false;          // a build stopped between its walk (which adds into d_bsum) and the
                                      // scan (which zeroes it again): the next build clears it first
    uint4 *d_scr = nullptr;                        // stream walk: staged events / offsets per range, overflow flags
    uint2 *d_scrh = nullptr;
    uint32_t *d_ovf = nullptr;
    uint2 *d_cnt = nullptr;           // [n_reads] lane-per-read census -> emit (svt_index2.inc)
    uint32_t n_groups = 0;            // 64-read groups of the lane-per-read index
    int ix_mode = 0;                  // index build: 0 by read length, 1 lane per read (svt_index2.inc), 2 stream
                                      // walk (svt_index.inc) -- SVTREK_IX=auto|lane|stream
    uint64_t *d_tot = nullptr;
    uint64_t n_evD = 0, n_evI = 0;
    // allele-consensus mode (svt_load_insseq / svt_poa_consensus)
    uint64_t *d_ins_off = nullptr;
    uint8_t *d_ins_bases = nullptr;
    bool insseq_loaded = false;
    PoaPool poa_small, poa_big;       // POA scratch slots (poa_pool)
    uint64_t poa_deferred = 0;        // loci the last svt_poa_consensus reran on full-size slots
    uint64_t *d_spoffD = nullptr, *d_spoffI = nullptr;   // span walk
    uint4 *d_spD = nullptr, *d_spI = nullptr;
    // the value-bucketed event index (svt_bucket.inc, svt_bucket_build.inc)
    bool bk_on = true;                // SVTREK_INDEX=lists: off (the span lists alone, rounds 1-5)
    bool bk_ready = false;            // built for the loaded pileup
    uint64_t bk_n = 0;                // buckets per array (every contig's)
    uint32_t *d_bkoff = nullptr;      // [BA_N][bk_n + 1] extents (indices into d_bkev)
    uint32_t *d_bkcur = nullptr;      // [BA_N][bk_n + 1] cursors of direct builds (k * count before build k)
    uint32_t *d_bkcap = nullptr;      // [BA_N][bk_n + 1] cursors of captured builds (zeroed by the graph)
    int32_t *d_bkpm = nullptr;        // [3][bk_n + 1] prefix max of the BELOW keys
    uint4 *d_bkev = nullptr;          // every array's events
    uint64_t bk_events[BA_N] = {};
    uint64_t *d_bkbase = nullptr;     // [n_targets] first bucket of contig t
    uint32_t *d_bknb = nullptr;       // [n_targets] its buckets
    uint32_t *d_bkmaxd = nullptr;     // [n_targets] its longest D > 50 op
    uint32_t bk_builds = 0;           // filing passes so far (the cursors' epoch)
    uint32_t bk_nev = 0;              // d_bkev's events (every array's)
    uint64_t dev_bytes = 0;
    bool loaded = false;
    svt_load_stats load_stats{};      // timings of the last svt_load_pileup
    // batch scratch
    svt_locus *d_loci = nullptr;
    svt_result *d_out = nullptr;
    size_t batch_cap = 0;
    // spill pool + status + work counters
    int32_t *d_pool = nullptr;
    unsigned long long pool_words = 0;
    unsigned char *d_ctl = nullptr;   // [0,8) pool head (epoch-tagged), [8,12) sticky status, [12,16) index
                                      // build guard, [16,16+8*W_N) work, [CTL_REDO, +16) left-over counters
    uint32_t epoch = 0;               // launches so far (pool epochs cycle through 1 .. 2^24-1)
    // launches run in submission order across streams (order_on)
    hipStream_t last_stream = nullptr;
    bool have_last = false;
    hipEvent_t order_ev = nullptr;
    // svt_open_multi: the contexts of devices[1..] (this one drives devices[0])
    std::vector<svt_ctx *> subs;
    // BGZF inflate (svt_bgzf_inflate): device buffers grown on demand, never shrunk
    uint8_t *d_infc = nullptr, *d_info = nullptr;
    svt_bgzf_block *d_infb = nullptr;
    uint32_t *d_inferr = nullptr;
    size_t infc_cap = 0, info_cap = 0, infb_cap = 0;
    double inf_ms = 0;                // device time of the last svt_bgzf_inflate's kernel
};

namespace {

svt_status fail(svt_ctx *c, svt_status code, const char *fmt, const char *detail) {
    if (c) snprintf(c->err, sizeof c->err, fmt, detail ? detail : "");
    return code;
}

#define HIP_TRY(ctx, expr)                                                               \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) return fail((ctx), SVT_EDEVICE, #expr ": %s", hipGetErrorString(e_)); \
    } while (0)

template <typename T>
void hfree(T *&p) {
    if (p) (void)hipFree((void *)p);
    p = nullptr;
}

// Every entry point runs on its context's device and gives the calling thread its current
// device back (one host thread may drive contexts on several GPUs).
struct DevGuard {
    int prev = -1, dev;
    bool ok = true;
    explicit DevGuard(int d) : dev(d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DevGuard() {
        if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
    }
};
#define DEV_GUARD(ctx)                                                                    \
    DevGuard dg_((ctx)->device);                                                          \
    if (!dg_.ok) return fail((ctx), SVT_EDEVICE, "hipSetDevice(%s) failed", "ctx device")

// A context's launches share its spill pool (epoch-tagged head), sticky status and work
// counters, so they must not overlap: a launch on another stream than the previous one
// first waits for everything issued so far on that one.
svt_status order_on(svt_ctx *c, hipStream_t st) {
    if (c->have_last && st != c->last_stream) {
        if (!c->order_ev) HIP_TRY(c, hipEventCreateWithFlags(&c->order_ev, hipEventDisableTiming));
        HIP_TRY(c, hipEventRecord(c->order_ev, c->last_stream));
        HIP_TRY(c, hipStreamWaitEvent(st, c->order_ev, 0));
    }
    c->last_stream = st;
    c->have_last = true;
    return SVT_OK;
}

// After a launch reported the spill pool exhausted: the head word of that launch's epoch
// holds every word its spilled windows asked for (svt_refine_*'s CAS adds them even past
// the end); grow the pool to that, at least doubling it.
svt_status grow_pool(svt_ctx *c) {
    unsigned long long head = 0;
    HIP_TRY(c, hipDeviceSynchronize());
    HIP_TRY(c, hipMemcpy(&head, c->d_ctl, 8, hipMemcpyDeviceToHost));
    const uint64_t need = (uint32_t)(head >> 40) == c->epoch ? (head & ((1ull << 40) - 1ull)) : 0ull;
    const uint64_t words = std::max<uint64_t>(need + need / 8 + 1024, 2 * c->pool_words);
    hfree(c->d_pool);
    c->pool_words = 0;
    if (hipMalloc(&c->d_pool, words * 4) != hipSuccess) {
        c->d_pool = nullptr;
        return fail(c, SVT_ENOMEM, "%s", "growing the candidate spill pool failed");
    }
    c->pool_words = words;
    return SVT_OK;
}

void free_pileup(svt_ctx *c) {
    hfree(c->d_pos); hfree(c->d_emax); hfree(c->d_rec); hfree(c->d_clip8); hfree(c->d_off64);
    hfree(c->d_tid_off); hfree(c->d_bkt_off); hfree(c->d_bkt); hfree(c->d_cigar);
    hfree(c->d_ins_off); hfree(c->d_ins_bases);
    hfree(c->d_part); hfree(c->d_cnt); hfree(c->d_agg); hfree(c->d_bsum); hfree(c->d_bpre); hfree(c->d_tot);
    hfree(c->d_scr); hfree(c->d_scrh); hfree(c->d_ovf);
    hfree(c->d_spoffD); hfree(c->d_spoffI); hfree(c->d_spD); hfree(c->d_spI);
    hfree(c->d_bkoff); hfree(c->d_bkcur); hfree(c->d_bkcap); hfree(c->d_bkev); hfree(c->d_bkpm);
    for (int A = 0; A < BA_N; A++) c->bk_events[A] = 0;
    hfree(c->d_bkbase); hfree(c->d_bknb); hfree(c->d_bkmaxd);
    c->bk_ready = false; c->bk_n = 0; c->bk_builds = 0; c->bk_nev = 0;
    c->insseq_loaded = false; c->n_ins = 0; c->n_ranges = 0;
    c->n_evD = c->n_evI = 0;
    c->loaded = false; c->dev_bytes = 0; c->n_reads = 0; c->n_ops = 0; c->n_targets = 0;
}

KArgs make_args(svt_ctx *c, const svt_locus *d_loci, svt_result *d_out, uint32_t n, bool count) {
    KArgs a;
    a.pile = DevPileup{c->d_pos, c->d_emax, c->d_rec, c->d_off64, c->d_tid_off, c->d_bkt_off, c->d_bkt,
                       c->d_cigar, c->d_spoffD, c->d_spoffI, c->d_spD, c->d_spI, c->n_targets};
    const svt_params &q = c->prm;
    // KParams::sent_ok: narrow + 2 >= max(range + max(ci, 0), 26) (64-bit: any int32 parameters)
    const int64_t width = std::max<int64_t>((int64_t)q.consensus_interval_range + std::max<int64_t>(q.consensus_interval, 0),
                                            SV_MIN_LENGTH / 2 + 1);
    a.prm = KParams{q.wider_interval, q.median_interval, q.narrow_interval, q.consensus_interval_range,
                    q.consensus_interval, q.consensus_min_count, 0, 0, (int64_t)q.narrow_interval + 2 >= width ? 1 : 0};
    a.loci = d_loci;
    a.out = d_out;
    a.n = n;
    a.pool = c->d_pool;
    a.pool_head = (unsigned long long *)c->d_ctl;
    a.pool_words = c->pool_words;
    a.epoch = c->epoch;
    a.status = (int32_t *)(c->d_ctl + 8);
    a.work = count ? (unsigned long long *)(c->d_ctl + 16) : nullptr;
    a.sw_sub = nullptr;
    a.sw_out = nullptr;
    a.rec_out = nullptr;
    a.rec_index = nullptr;
    a.rec_base = 0;
    a.redo_list = nullptr;
    a.redo_ctr = a.redo_next = nullptr;
    a.bk.ev = c->d_bkev;
    a.bk.off = c->d_bkoff;
    a.bk.pm = c->d_bkpm;
    a.bk.nbk = c->bk_n;
    a.bk.cbase = c->d_bkbase;
    a.bk.cnb = c->d_bknb;
    a.bk.maxd = c->d_bkmaxd;
    a.bk.on = c->bk_ready ? 1 : 0;
    return a;
}

svt_status launch(svt_ctx *c, const svt_locus *d_loci, svt_result *d_out, size_t n, hipStream_t st, bool count,
                  svt_record *rec_out = nullptr, const uint32_t *rec_index = nullptr, uint32_t rec_base = 0) {
    if (n == 0) return SVT_OK;
    if (n > 0x3fffffffull) return fail(c, SVT_EINVAL, "batch too large (%s)", "n > 2^30-1");
    svt_status s = order_on(c, st);
    if (s) return s;
    // A launch captured into a HIP graph (the caller's stream capture) is replayed with the
    // epoch and redo-counter parity of its capture, so its graph also clears the pool head and
    // its redo counter itself (two memset nodes); otherwise nothing per launch is reset.
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (st) HIP_TRY(c, hipStreamIsCapturing(st, &cap));
    const bool captured = cap == hipStreamCaptureStatusActive;
    // no per-launch reset of the spill pool (epoch-tagged head; launches never overlap,
    // order_on); the work counters of a counting launch start from zero; the head word is
    // cleared once per epoch cycle
    c->epoch = c->epoch % ((1u << 24) - 1u) + 1u;
    if (c->epoch == 1 || captured) {   // a new epoch cycle (or every replay): the pool head starts from zero
        HIP_TRY(c, hipMemsetAsync(c->d_ctl, 0, 8, st));
    }
    if (count) HIP_TRY(c, hipMemsetAsync(c->d_ctl + 16, 0, 8 * W_N, st));
    KArgs a = make_args(c, d_loci, d_out, (uint32_t)n, count);
    a.rec_out = reinterpret_cast<uint4 *>(rec_out);
    a.rec_index = rec_index;
    a.rec_base = rec_base;
    dim3 grid((unsigned)((2 * n + WPB - 1) / WPB)), block(64 * WPB);
    if (count) {
        hipLaunchKernelGGL((refine_kernel<true, G_SPAN>), grid, block, 0, st, a);
    } else if (c->lane_vote && (c->lane_w != 0 || 2 * n >= (size_t)65536)) {
        // lane kernel (32 windows a wave) once the batch has >= 64K windows; below that the
        // one-wave-per-window span kernel is as fast or faster (fewer, longer waves leave the
        // chip underfilled: cfg2 20K windows 33 us span vs 76 us lane<8>, 107 us lane<32>;
        // cfg3 100K windows 111 vs 109 us; cfg4 2M windows 2.23 ms vs 0.905 ms)
        if (c->redo_cap < 2 * n) {   // window list of the wave-wide left-overs (grown, never shrunk)
            hfree(c->d_redo);
            c->redo_cap = 0;
            HIP_TRY(c, hipMalloc(&c->d_redo, 2 * n * sizeof(uint32_t)));
            c->redo_cap = 2 * n;
        }
        // Two left-over counters alternate between direct lane launches: this launch appends to
        // ctr[par]; its redo kernel reads that and zeroes ctr[par ^ 1] for the next one.  The
        // parity advances on direct lane launches only (counting and span launches in between leave
        // both alone), and both start zeroed (svt_open).  A launch captured into a graph has its own
        // counter, ctr[2], zeroed by a memset node at the head of its graph, and its redo kernel's
        // "next" word is the scratch ctr[3]: replays run whenever the caller likes, so they must
        // neither read nor leave state the direct launches' alternation depends on.
        a.redo_list = c->d_redo;
        uint32_t *ctr = (uint32_t *)(c->d_ctl + CTL_REDO);
        if (captured) {
            a.redo_ctr = ctr + 2;
            a.redo_next = ctr + 3;
            HIP_TRY(c, hipMemsetAsync(a.redo_ctr, 0, sizeof(uint32_t), st));
        } else {
            a.redo_ctr = ctr + c->lane_par;
            a.redo_next = ctr + (c->lane_par ^ 1u);
            c->lane_par ^= 1u;
        }
        // (16 windows a wave for the 250K-window launches of a 125K-locus shard measured slower:
        // 0.132-0.138 vs 0.117-0.121 ms, profiles/r04_sh)
        const dim3 lgrid((unsigned)((2 * n + WPB * 32 - 1) / (WPB * 32)));
        if (c->bk_ready) hipLaunchKernelGGL((refine_lane_kernel<32, true>), lgrid, block, 0, st, a);
        else hipLaunchKernelGGL((refine_lane_kernel<32, false>), lgrid, block, 0, st, a);
        hipLaunchKernelGGL(refine_redo_kernel, dim3(8192), block, 0, st, a);   // ~1 left-over window per wave
    } else {
        hipLaunchKernelGGL(refine_span_kernel, grid, block, 0, st, a);
    }
    HIP_TRY(c, hipGetLastError());
    return SVT_OK;
}

svt_status ensure_batch(svt_ctx *c, size_t n) {
    if (n <= c->batch_cap) return SVT_OK;
    hfree(c->d_loci); hfree(c->d_out);
    c->batch_cap = 0;
    HIP_TRY(c, hipMalloc(&c->d_loci, n * sizeof(svt_locus)));
    HIP_TRY(c, hipMalloc(&c->d_out, n * sizeof(svt_result)));
    c->batch_cap = n;
    return SVT_OK;
}

template <typename T>
svt_status upload(svt_ctx *c, T *&dst, const T *src, size_t n, size_t pad_elems = 0) {
    size_t bytes = (n + pad_elems) * sizeof(T);
    HIP_TRY(c, hipMalloc(&dst, bytes ? bytes : sizeof(T)));
    if (n) HIP_TRY(c, hipMemcpy(dst, src, n * sizeof(T), hipMemcpyHostToDevice));
    if (pad_elems) HIP_TRY(c, hipMemset(dst + n, 0, pad_elems * sizeof(T)));
    c->dev_bytes += bytes;
    return SVT_OK;
}

// POA scratch, kept across calls: one slot per persistent wave in two pools.  The many
// small slots hold graphs up to POA_SMALL_NODES nodes with POA_SMALL_SPILL spill rows (a
// typical allele's graph is a few thousand nodes and spills none); loci that outgrow them
// rerun on the few full-size slots.  Sizes at the default parameters: 2560 x 8.6 MB
// (10 waves per CU: the LDS ring bounds occupancy at 11) and 256 x 50 MB.
#ifndef SVT_POA_SLOTS_SMALL
#define SVT_POA_SLOTS_SMALL 2560
#endif
constexpr uint64_t POA_SLOTS_SMALL = SVT_POA_SLOTS_SMALL;
constexpr uint64_t POA_SLOTS_BIG = 256;
constexpr int32_t POA_SMALL_NODES = 16384;
constexpr int32_t POA_SMALL_SPILL = 256;

svt_status poa_pool(svt_ctx *c, PoaPool &pl, int32_t node_cap, int32_t spill_cap, const svt_poa_params *p,
                    uint64_t want) {
    const uint64_t sb = poa_slot_bytes(node_cap, spill_cap, p->max_len);
    if (pl.d && pl.slot_bytes == sb && pl.nslots >= want) return SVT_OK;
    hfree(pl.d);
    pl.nslots = 0;
    if (hipMalloc(&pl.d, want * sb) != hipSuccess) {
        pl.d = nullptr;
        return fail(c, SVT_ENOMEM, "%s", "poa scratch (lower max_nodes / max_len)");
    }
    pl.slot_bytes = sb;
    pl.nslots = (uint32_t)want;
    return SVT_OK;
}

// SVTREK_POA_SMALL_NODES overrides the small slots' node budget (tests force deferral).
int32_t poa_small_cap(const svt_poa_params *p) {
    const char *ev = getenv("SVTREK_POA_SMALL_NODES");
    const int32_t want = ev ? (int32_t)atoi(ev) : POA_SMALL_NODES;
    return std::min(p->max_nodes, std::max(want, p->max_len + 2));
}

// One persistent launch of poa_kernel over d_list (or all n loci) on pool pl; synchronous.
svt_status poa_launch(svt_ctx *c, PoaArgs a, const PoaPool &pl, int32_t node_cap, int32_t spill_cap,
                      const uint32_t *d_list, uint32_t n, uint32_t *d_queue) {
    a.slots = pl.d;
    a.slot_bytes = pl.slot_bytes;
    a.node_cap = node_cap;
    a.spill_cap = spill_cap;
    a.list = d_list;
    a.n = n;
    a.queue = d_queue;
    a.diag = nullptr;
    HIP_TRY(c, hipMemset(d_queue, 0, sizeof(uint32_t)));
#if SVT_POA_DIAG
    HIP_TRY(c, hipMalloc(&a.diag, PD_N * sizeof(unsigned long long)));
    HIP_TRY(c, hipMemset(a.diag, 0, PD_N * sizeof(unsigned long long)));
    HIP_TRY(c, hipMemset(a.diag + PD_T0, 0xff, sizeof(unsigned long long)));
#endif
    const unsigned grid = (unsigned)std::min<uint64_t>(pl.nslots, n);
    hipLaunchKernelGGL(poa_kernel, dim3(grid), dim3(64), 0, nullptr, a);
    HIP_TRY(c, hipGetLastError());
    HIP_TRY(c, hipDeviceSynchronize());
#if SVT_POA_DIAG
    unsigned long long h[PD_N];
    HIP_TRY(c, hipMemcpy(h, a.diag, sizeof h, hipMemcpyDeviceToHost));
    (void)hipFree(a.diag);
    fprintf(stderr, "poa_diag node_cap=%d grid=%u loci=%u wave-ms: support %.1f load %.1f rows %.1f trace %.1f "
            "fuse %.1f cons %.1f | rows %llu steps %llu seqs %llu far %llu\n", node_cap, grid, n, h[PD_SUPPORT] * 1e-5,
            h[PD_LOAD] * 1e-5, h[PD_ROWS] * 1e-5, h[PD_TRACE] * 1e-5, h[PD_FUSE] * 1e-5, h[PD_CONS] * 1e-5,
            h[PD_NROWS], h[PD_NSTEPS], h[PD_NSEQ], h[PD_NFAR]);
    fprintf(stderr, "poa_diag span %.1f ms, longest locus %.1f ms, busiest wave %.1f ms\n",
            (h[PD_T1] - h[PD_T0]) * 1e-5, h[PD_LOCMAX] * 1e-5, h[PD_WAVEMAX] * 1e-5);
#endif
    return SVT_OK;
}

svt_status poa_run(svt_ctx *c, const svt_poa_params *p, const svt_locus *loci, const svt_result *refined, size_t n,
                   int32_t cap, uint8_t *bases, svt_poa_result *res) {
    svt_locus *d_loci = nullptr;
    svt_result *d_ref = nullptr;
    uint8_t *d_out = nullptr;
    int4 *d_res = nullptr;
    uint32_t *d_aux = nullptr;   // [0] work queue, [1 .. n] locus order, [n+1 .. 2n] cost estimates
    int32_t *d_sup = nullptr;    // [n] supporting sequences found, then [n][max_support] their indices
    svt_status s = SVT_OK;
    auto chk = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && s == SVT_OK) s = fail(c, SVT_EDEVICE, what, hipGetErrorString(e));
        return s == SVT_OK;
    };
    const int32_t small_cap = poa_small_cap(p);
    if (chk(hipMalloc(&d_loci, n * sizeof(svt_locus)), "hipMalloc: %s") &&
        chk(hipMalloc(&d_ref, n * sizeof(svt_result)), "hipMalloc: %s") &&
        chk(hipMalloc(&d_out, std::max<size_t>(1, n * (size_t)cap)), "hipMalloc: %s") &&
        chk(hipMalloc(&d_res, n * sizeof(int4)), "hipMalloc: %s") &&
        chk(hipMalloc(&d_aux, (2 * n + 1) * sizeof(uint32_t)), "hipMalloc: %s") &&
        chk(hipMalloc(&d_sup, n * (1 + (size_t)p->max_support) * sizeof(int32_t)), "hipMalloc: %s") &&
        chk(hipMemcpy(d_loci, loci, n * sizeof(svt_locus), hipMemcpyHostToDevice), "H2D: %s") &&
        chk(hipMemcpy(d_ref, refined, n * sizeof(svt_result), hipMemcpyHostToDevice), "H2D: %s")) {
        const KArgs k = make_args(c, nullptr, nullptr, 0, false);
        PoaArgs a;
        a.pile = k.pile;
        a.prm = k.prm;
        a.pp = PoaParams{p->match, p->mismatch, p->gap_open, p->gap_ext, p->band_b, p->band_f_permille,
                         p->max_seqs, p->max_len, p->max_nodes, p->support_radius, p->max_support};
        a.loci = d_loci;
        a.refined = d_ref;
        a.n = (uint32_t)n;
        a.ins_base = c->d_spoffI;
        a.ins_off = c->d_ins_off;
        a.ins_bases = c->d_ins_bases;
        a.cap = cap;
        a.out = d_out;
        a.res = d_res;
        a.nsupg = d_sup;
        a.supg = d_sup + n;
        a.est = d_aux + 1 + n;
        a.diag = nullptr;
        // supports + cost estimates, then the loci longest first (ties: input order)
        hipLaunchKernelGGL(poa_support_kernel, dim3((unsigned)std::min<size_t>(n, 8192)), dim3(64), 0, nullptr, a);
        std::vector<uint32_t> est(n), order(n);
        if (chk(hipGetLastError(), "poa_support_kernel: %s") &&
            chk(hipMemcpy(est.data(), a.est, n * sizeof(uint32_t), hipMemcpyDeviceToHost), "D2H: %s")) {
            for (size_t i = 0; i < n; i++) order[i] = (uint32_t)i;
            std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return est[x] > est[y]; });
            chk(hipMemcpy(d_aux + 1, order.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice), "H2D: %s");
        }
        if (s == SVT_OK)
            s = poa_pool(c, c->poa_small, small_cap, POA_SMALL_SPILL, p, std::min<uint64_t>(n, POA_SLOTS_SMALL));
        if (s == SVT_OK) s = poa_launch(c, a, c->poa_small, small_cap, POA_SMALL_SPILL, d_aux + 1, (uint32_t)n, d_aux);
        if (s == SVT_OK && chk(hipMemcpy(res, d_res, n * sizeof(int4), hipMemcpyDeviceToHost), "D2H: %s")) {
            std::vector<uint32_t> deferred;   // in the same longest-first order
            for (size_t q = 0; q < n; q++)
                if (res[order[q]].status == POA_DEFER) deferred.push_back(order[q]);
            if (!deferred.empty()) {
                const uint32_t nd = (uint32_t)deferred.size();
                if (chk(hipMemcpy(d_aux + 1, deferred.data(), nd * sizeof(uint32_t), hipMemcpyHostToDevice), "H2D: %s"))
                    s = poa_pool(c, c->poa_big, p->max_nodes, p->max_nodes + 2, p, std::min<uint64_t>(nd, POA_SLOTS_BIG));
                if (s == SVT_OK) s = poa_launch(c, a, c->poa_big, p->max_nodes, p->max_nodes + 2, d_aux + 1, nd, d_aux);
                if (s == SVT_OK) chk(hipMemcpy(res, d_res, n * sizeof(int4), hipMemcpyDeviceToHost), "D2H: %s");
            }
            c->poa_deferred = deferred.size();
            if (s == SVT_OK && cap > 0) chk(hipMemcpy(bases, d_out, n * (size_t)cap, hipMemcpyDeviceToHost), "D2H: %s");
        }
    }
    hfree(d_loci); hfree(d_ref); hfree(d_out); hfree(d_res); hfree(d_aux); hfree(d_sup);
    return s;
}

}  // namespace

extern "C" {

const char *svt_version(void) { return SVT_VERSION; }

const char *svt_last_error(const svt_ctx *ctx) { return ctx ? ctx->err : "null context"; }

svt_status svt_open(const svt_params *params, int device, svt_ctx **out) {
    if (!params || !out) return SVT_EINVAL;
    *out = nullptr;
    if (params->consensus_min_count < 1) return SVT_EINVAL;   // min_count <= 0 reads locations[-1]
    svt_ctx *c = new (std::nothrow) svt_ctx();
    if (!c) return SVT_ENOMEM;
    c->prm = *params;
    const char *g = getenv("SVTREK_GATHER");   // "span1": the one-wave-per-window kernel at every batch size
    c->lane_vote = !(g && strcmp(g, "span1") == 0);
    if (const char *x = getenv("SVTREK_IX")) c->ix_mode = strcmp(x, "lane") == 0 ? 1 : strcmp(x, "stream") == 0 ? 2 : 0;
    if (const char *x = getenv("SVTREK_IX_RANGES")) c->ix_ranges = std::max<uint64_t>(1, strtoull(x, nullptr, 10));
    if (const char *lw = getenv("SVTREK_LANE_W")) c->lane_w = atoi(lw) == 32 ? 32 : 0;
    if (const char *x = getenv("SVTREK_INDEX")) c->bk_on = strcmp(x, "lists") != 0;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
        delete c;
        return SVT_EDEVICE;
    }
    if (device >= 0) {
        if (device >= ndev) { delete c; return SVT_EDEVICE; }
        c->device = device;
    } else {
        (void)hipGetDevice(&c->device);
    }
    DevGuard dg(c->device);
    if (!dg.ok) { delete c; return SVT_EDEVICE; }
    uint64_t pool_bytes = params->spill_bytes ? params->spill_bytes : (64ull << 20);
    c->pool_words = pool_bytes / 4;
    if (hipMalloc(&c->d_pool, c->pool_words * 4) != hipSuccess || hipMalloc(&c->d_ctl, CTL_BYTES) != hipSuccess) {
        hfree(c->d_pool);
        delete c;
        return SVT_ENOMEM;
    }
    (void)hipMemset(c->d_ctl, 0, CTL_BYTES);
    // load the code object now (HIP loads it lazily at the first launch), so that no later
    // call -- and no timing of one -- pays for it
    hipFuncAttributes fa;
    (void)hipFuncGetAttributes(&fa, reinterpret_cast<const void *>(index_kernel));
    *out = c;
    return SVT_OK;
}

svt_status svt_open_multi(const svt_params *params, int device_count, const int *devices, svt_ctx **out) {
    if (!params || !out || device_count < 1) return SVT_EINVAL;
    *out = nullptr;
    svt_ctx *c = nullptr;
    svt_status s = svt_open(params, devices ? devices[0] : 0, &c);
    if (s) return s;
    for (int i = 1; i < device_count; i++) {
        svt_ctx *d = nullptr;   // (a device may repeat: two independent contexts on one GPU)
        s = svt_open(params, devices ? devices[i] : i, &d);
        if (s) {
            svt_close(c);
            return s;
        }
        c->subs.push_back(d);
    }
    *out = c;
    return SVT_OK;
}

int svt_device_count(const svt_ctx *c) { return c ? 1 + (int)c->subs.size() : 0; }

extern "C++" {
namespace {

// Run fn(k) for k = 0 .. n-1 on up to `cap` threads (the host pass of svt_load_pileup is per contig).
template <typename F>
void parallel_for(size_t n, size_t cap, F fn) {
    const size_t T = std::max<size_t>(1, std::min<size_t>({n, cap, (size_t)std::max(1u, std::thread::hardware_concurrency())}));
    if (T <= 1) {
        for (size_t k = 0; k < n; k++) fn(k);
        return;
    }
    std::atomic<size_t> next{0};
    std::vector<std::thread> th;
    for (size_t t = 0; t < T; t++)
        th.emplace_back([&] {
            for (size_t k; (k = next.fetch_add(1)) < n;) fn(k);
        });
    for (auto &x : th) x.join();
}

// The device index of the loaded pileup (svt_index.inc / svt_index2.inc).  Stream walk: the walk
// (one pass over the stream, events staged per range), an exclusive scan of the range totals, the
// staged rows to their places.  Lane per read: census, the scan of the group totals, emit.
// `first`: between scan and placement, size and allocate the event lists from the totals (one
// synchronous read-back); later calls (svt_reindex) reuse them -- the totals depend on the
// pileup only.  `ms`: the index kernels' device time (HIP events; read-back and allocations
// excluded).
// lane per read (svt_index2.inc) for short reads -- a wave's 64 reads then take a few steps
// each; long reads (a lane walking thousands of ops waits on its loads) take the stream walk,
// which spreads every slot of 256 ops over the wave; never for a group of > 2^27 ops
bool index_lane(const svt_ctx *c, uint64_t nops, uint64_t nreads) {
    return c->n_groups > 0 && (c->ix_mode == 1 || (c->ix_mode == 0 && nops <= 64ull * nreads));
}

IxArgs ix_args(const svt_ctx *c) {
    IxArgs a;
    a.stream = c->d_cigar;
    a.soff = c->d_off64;
    a.rec = c->d_rec;
    a.clip8 = c->d_clip8;
    a.part = c->d_part;
    a.agg = c->d_agg;
    a.bsum = c->d_bsum;
    a.bpre = c->d_bpre;
    a.spoffD = c->d_spoffD;
    a.spoffI = c->d_spoffI;
    a.spD = c->d_spD;
    a.spI = c->d_spI;
    a.capD = c->n_evD;
    a.capI = c->n_evI;
    a.err = (uint32_t *)(c->d_ctl + 12);   // sticky status word 2 (svt_sync reports it)
    a.scr = c->d_scr;
    a.scrh = c->d_scrh;
    a.ovf = c->d_ovf;
    a.n_ranges = c->n_ranges;
    return a;
}

svt_status build_index(svt_ctx *c, hipStream_t st, bool first, double *ms) {
    IxArgs a = ix_args(c);
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    if (ms)
        for (auto &e : ev) HIP_TRY(c, hipEventCreate(&e));
    auto done = [&](svt_status r) {
        for (auto &e : ev)
            if (e) (void)hipEventDestroy(e);
        return r;
    };
    const bool lane = index_lane(c, c->n_ops, (uint64_t)c->n_reads);
    c->load_stats.index_kind = lane ? 1u : 2u;
    const uint32_t nparts = lane ? c->n_groups : c->n_ranges;   // what the scan runs over
    Ix2Args a2{a, c->d_cnt, (uint64_t)c->n_reads, c->n_groups};
    const dim3 grid2((unsigned)((c->n_groups + IX2_WPB - 1) / IX2_WPB)), block2(64 * IX2_WPB);
    const dim3 grid1((unsigned)((c->n_ranges + IX_WPB - 1) / IX_WPB)), block1(64 * IX_WPB);
    if (ms && hipEventRecord(ev[0], st) != hipSuccess) return done(fail(c, SVT_EDEVICE, "%s", "hipEventRecord"));
    if (c->bsum_dirty) {
        if (hipMemsetAsync(c->d_bsum, 0, c->n_bsum * sizeof(IxTot), st) != hipSuccess)
            return done(fail(c, SVT_EDEVICE, "%s", "index block sums: hipMemsetAsync"));
        c->bsum_dirty = false;
    }
    c->bsum_dirty = true;
    if (lane)
        hipLaunchKernelGGL(ix2_census_kernel, grid2, block2, 0, st, a2);
    else
        hipLaunchKernelGGL(index_kernel, grid1, block1, 0, st, a);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) {   // the blocks' exclusive prefixes (ix_part_base adds the ranges' within a block)
        hipLaunchKernelGGL(ix_scan_blocks_kernel, dim3(1), dim3(IX_SCAN_T), 0, st, c->d_bsum, c->d_bpre,
                           (nparts + IX_BLK - 1) / IX_BLK, c->d_tot, c->d_spoffD, c->d_spoffI, (uint64_t)c->n_reads);
        e = hipGetLastError();
    }
    if (e != hipSuccess) return done(fail(c, SVT_EDEVICE, "index census: %s", hipGetErrorString(e)));
    c->bsum_dirty = false;   // the scan launched: it zeroes the block sums behind itself
    if (ms && hipEventRecord(ev[1], st) != hipSuccess) return done(fail(c, SVT_EDEVICE, "%s", "hipEventRecord"));
    if (first) {
        uint64_t t[IX_NTOT];
        e = hipMemcpyAsync(t, c->d_tot, sizeof t, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return done(fail(c, SVT_EDEVICE, "index totals: %s", hipGetErrorString(e)));
        c->n_evD = t[IX_D];
        c->n_evI = t[IX_I];
        c->n_ins = t[IX_I];
        svt_status s;
        if ((s = upload<uint4>(c, c->d_spD, nullptr, 0, std::max<uint64_t>(c->n_evD, 1)))) return done(s);
        if ((s = upload<uint4>(c, c->d_spI, nullptr, 0, std::max<uint64_t>(c->n_evI, 1)))) return done(s);
        a.spD = c->d_spD;
        a.spI = c->d_spI;
        a.capD = c->n_evD;
        a.capI = c->n_evI;
        a2.a = a;
    }
    if (ms && hipEventRecord(ev[2], st) != hipSuccess) return done(fail(c, SVT_EDEVICE, "%s", "hipEventRecord"));
    if (lane) hipLaunchKernelGGL(ix2_emit_kernel, grid2, block2, 0, st, a2);
    else hipLaunchKernelGGL(ix_copy_kernel, grid1, block1, 0, st, a);
    e = hipGetLastError();
    if (e != hipSuccess) return done(fail(c, SVT_EDEVICE, "index emit: %s", hipGetErrorString(e)));
    if (ms) {
        float t0 = 0.f, t1 = 0.f;
        e = hipEventRecord(ev[3], st);
        if (e == hipSuccess) e = hipEventSynchronize(ev[3]);
        if (e == hipSuccess) e = hipEventElapsedTime(&t0, ev[0], ev[1]);
        if (e == hipSuccess) e = hipEventElapsedTime(&t1, ev[2], ev[3]);
        if (e != hipSuccess) return done(fail(c, SVT_EDEVICE, "index timing: %s", hipGetErrorString(e)));
        *ms = (double)t0 + (double)t1;
    }
    return done(SVT_OK);
}

// ---- the value-bucketed event index (svt_bucket_build.inc): launch arguments, one pass, the
// first build at load
BkBuild bk_args(const svt_ctx *c, bool count, bool captured) {
    BkBuild b{};
    b.ev = c->d_bkev;
    b.off = c->d_bkoff;
    b.cur = count ? c->d_bkoff : captured ? c->d_bkcap : c->d_bkcur;
    b.pmx = c->d_bkpm;
    b.nbk = c->bk_n;
    b.maxd = c->d_bkmaxd;
    b.cbase = c->d_bkbase;
    b.cnb = c->d_bknb;
    b.k = count || captured ? 0u : c->bk_builds;
    b.n_ev = c->bk_nev;
    b.err = (uint32_t *)(c->d_ctl + 12);   // sticky status word 2 (svt_sync reports it)
    return b;
}

// One counting or filing pass on st: short reads walked from the CIGAR stream, long reads filed
// from the span lists (which the caller rebuilt first).
svt_status bk_pass(svt_ctx *c, hipStream_t st, bool count, bool captured) {
    const IxArgs a = ix_args(c);
    const BkBuild b = bk_args(c, count, captured);
    const uint64_t nr = (uint64_t)c->n_reads;
    if (index_lane(c, c->n_ops, nr)) {
        const dim3 grid((unsigned)((c->n_groups + IXB_WPB - 1) / IXB_WPB)), block(64 * IXB_WPB);
        if (count) hipLaunchKernelGGL(ixb_lane_kernel<true>, grid, block, 0, st, a, b, nr);
        else hipLaunchKernelGGL(ixb_lane_kernel<false>, grid, block, 0, st, a, b, nr);
    } else if (count) {   // (at load: the span lists the first build made)
        const dim3 grid((unsigned)((nr + IXB_T - 1) / IXB_T)), block(IXB_T);
        hipLaunchKernelGGL(ixb_lists_kernel<true>, grid, block, 0, st, a, b, nr);
    } else {              // from the stream walk's stage (index_kernel ran just before on st)
        const dim3 grid((unsigned)((c->n_ranges + IX_WPB - 1) / IX_WPB)), block(64 * IX_WPB);
        hipLaunchKernelGGL(ixb_copy_kernel, grid, block, 0, st, a, b);
    }
    HIP_TRY(c, hipGetLastError());
    return SVT_OK;
}

svt_status bk_check_err(svt_ctx *c) {
    uint32_t e = 0;
    HIP_TRY(c, hipDeviceSynchronize());
    HIP_TRY(c, hipMemcpy(&e, c->d_ctl + 12, 4, hipMemcpyDeviceToHost));
    if (e) {
        HIP_TRY(c, hipMemset(c->d_ctl + 12, 0, 4));
        return fail(c, SVT_EDEVICE, "%s", "device index build: the value buckets disagree with their count");
    }
    return SVT_OK;
}

// The first build (svt_load_pileup, after the span lists): buckets per contig from the largest
// pos / endpos (values past them -- walks lengthened by H / P / N ops -- share the contig's last
// bucket), the counting pass, the extents and prefix maxima on the host, the filing pass.  A pileup
// whose events or buckets pass 2^32 keeps the span lists alone (bk_ready stays false).
svt_status bk_load(svt_ctx *c, const std::vector<int64_t> &vtop) {
    const int32_t nt = c->n_targets;
    std::vector<uint64_t> cbase((size_t)nt);
    std::vector<uint32_t> cnb((size_t)nt);
    uint64_t NB = 0;
    for (int32_t t = 0; t < nt; t++) {
        const uint64_t nb = (((uint64_t)std::max<int64_t>(vtop[(size_t)t], 0) + 65536u) >> BKS) + 2u;
        cbase[(size_t)t] = NB;
        cnb[(size_t)t] = (uint32_t)nb;
        NB += nb;
    }
    if (nt == 0 || NB >= 0xffffffffull) return SVT_OK;
    svt_status s;
    if ((s = upload(c, c->d_bkbase, cbase.data(), cbase.size()))) return s;
    if ((s = upload(c, c->d_bknb, cnb.data(), cnb.size()))) return s;
    if ((s = upload<uint32_t>(c, c->d_bkmaxd, nullptr, 0, (size_t)nt))) return s;
    const uint64_t S1 = NB + 1;   // the tables' stride per array
    if ((s = upload<uint32_t>(c, c->d_bkoff, nullptr, 0, BA_N * S1))) return s;   // (zeroed: the counts)
    if ((s = upload<uint32_t>(c, c->d_bkcur, nullptr, 0, BA_N * S1))) return s;
    if ((s = upload<uint32_t>(c, c->d_bkcap, nullptr, 0, (BA_N * S1 + 3) / 4 * 4))) return s;   // (whole uint4s: bk_zero_kernel)
    if ((s = upload<int32_t>(c, c->d_bkpm, nullptr, 0, 3 * S1))) return s;
    HIP_TRY(c, hipMemset(c->d_bkpm, 0xff, 3 * S1 * sizeof(int32_t)));   // -1: no key
    c->bk_n = NB;
    if ((s = bk_pass(c, nullptr, true, false)) || (s = bk_check_err(c))) return s;
    // the extents: every array's buckets in order, the arrays one after the other in d_bkev
    std::vector<uint32_t> cnt((size_t)(BA_N * S1));
    std::vector<int32_t> pm((size_t)(3 * S1));
    HIP_TRY(c, hipMemcpy(cnt.data(), c->d_bkoff, cnt.size() * 4, hipMemcpyDeviceToHost));
    HIP_TRY(c, hipMemcpy(pm.data(), c->d_bkpm, pm.size() * 4, hipMemcpyDeviceToHost));
    uint64_t acc = 0;
    for (int A = 0; A < BA_N; A++) {
        const uint64_t a0 = acc;
        uint32_t *o = cnt.data() + (size_t)A * S1;
        for (uint64_t g = 0; g < NB; g++) {
            const uint32_t x = o[(size_t)g];
            o[(size_t)g] = (uint32_t)acc;
            acc += x;
            if (acc >= 0xffffffffull) return SVT_OK;   // (bk_ready stays false: the span lists alone)
        }
        o[(size_t)NB] = (uint32_t)acc;
        c->bk_events[A] = acc - a0;
        if (A < 3)   // the BELOW keys' prefix maxima, within each contig
            for (int32_t t = 0; t < nt; t++) {
                int32_t m = -1;
                int32_t *q = pm.data() + (size_t)A * S1;
                for (uint64_t g = cbase[(size_t)t], g1 = g + cnb[(size_t)t]; g < g1; g++) m = q[(size_t)g] = std::max(m, q[(size_t)g]);
            }
    }
    HIP_TRY(c, hipMemcpy(c->d_bkoff, cnt.data(), cnt.size() * 4, hipMemcpyHostToDevice));
    HIP_TRY(c, hipMemcpy(c->d_bkpm, pm.data(), pm.size() * 4, hipMemcpyHostToDevice));
    if ((s = upload<uint4>(c, c->d_bkev, nullptr, 0, std::max<uint64_t>(acc, 1)))) return s;
    c->bk_nev = (uint32_t)acc;
    c->bk_builds = 0;   // the cursors are zero: the first filing pass is epoch 0
    if ((s = bk_pass(c, nullptr, false, false)) || (s = bk_check_err(c))) return s;
    c->bk_builds = 1;
    c->bk_ready = true;
    return SVT_OK;
}

}  // namespace
}  // extern "C++"

// The pileup of a context from per-read columns in host memory -- nc[r] = n_cigar | clip << 30,
// soff[0..nr] the reads' offsets in the CIGAR stream (a read without ops owns one 0M word) --
// and the stream itself, in host memory (stream_h) or already on the device (stream_d, with
// STREAM_PAD zero words after its end: adopted, the context frees it).  The host pass
// validates and builds the prefix-max endpos, the records, the read buckets, the index ranges;
// then the uploads and the first device index build.
static svt_status load_core(svt_ctx *c, int32_t nt, const int64_t *tid_off, const int32_t *pos, const int32_t *endpos,
                            const uint32_t *nc, const uint64_t *soff, const uint32_t *stream_h, uint32_t *stream_d,
                            uint64_t nops, double t_pre_ms) {
    using clk = std::chrono::steady_clock;
    auto ms_since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
    const clk::time_point t_start = clk::now();
    const int64_t nr = nt ? tid_off[nt] : 0;
    const uint64_t nstream = nr > 0 ? soff[nr] : 0;
    // ---- host pass, per contig in parallel: validation, prefix-max endpos, records, buckets
    std::vector<int32_t> emax((size_t)nr);
    std::vector<uint4> rec((size_t)nr);
    std::vector<std::vector<uint2>> bk((size_t)nt);
    std::vector<const char *> bad((size_t)nt, nullptr);
    std::vector<int64_t> vtop((size_t)nt, 0);   // per contig its largest pos / endpos (the value buckets)
    parallel_for((size_t)nt, 16, [&](size_t t) {
        const int64_t r0 = tid_off[t], r1 = tid_off[t + 1];
        if (r1 - r0 > 0xffffffffll) { bad[t] = "> 2^32 reads on one contig"; return; }
        int32_t m = INT32_MIN, maxpos = 0;
        for (int64_t r = r0; r < r1; r++) {
            if (r > r0 && pos[r] < pos[r - 1]) { bad[t] = "reads not sorted by pos within a contig"; return; }
            if (pos[r] < 0 || endpos[r] <= pos[r]) { bad[t] = "pos < 0 or endpos <= pos"; return; }
            const uint64_t w = soff[r + 1] - soff[r], n = nc[r] & NCIG_MASK;
            if (soff[r + 1] < soff[r] || soff[r + 1] > nstream || w != std::max<uint64_t>(n, 1)) {
                bad[t] = "bad cig_off";
                return;
            }
            if (endpos[r] > m) m = endpos[r];
            maxpos = std::max(maxpos, pos[r]);
            emax[(size_t)r] = m;
            rec[(size_t)r] = make_uint4((uint32_t)pos[r], (uint32_t)endpos[r], nc[r], (uint32_t)t);   // .w: the contig
        }
        // bucket b = 0..nb-1: {first contig-relative read with pos >= b << BKT_SHIFT, first with
        // emax >= b << BKT_SHIFT}; the last bucket lies past every pos and endpos: {nr, nr}
        const int64_t top = r1 > r0 ? std::max<int64_t>(maxpos, m) : 0;
        vtop[t] = top;
        const int64_t nb = (top >> BKT_SHIFT) + 2;
        std::vector<uint2> &B = bk[t];
        B.reserve((size_t)nb);
        int64_t rp = r0, re = r0;
        for (int64_t b = 0; b < nb; b++) {
            const int64_t x = b << BKT_SHIFT;
            while (rp < r1 && (int64_t)pos[rp] < x) rp++;
            while (re < r1 && (int64_t)emax[(size_t)re] < x) re++;
            B.push_back(make_uint2((uint32_t)(rp - r0), (uint32_t)(re - r0)));
        }
    });
    for (int32_t t = 0; t < nt; t++)
        if (bad[(size_t)t]) return fail(c, SVT_EINVAL, "pileup: %s", bad[(size_t)t]);
    if (stream_d) c->d_cigar = stream_d;   // the context owns it from here on (freed with the pileup)
    std::vector<int64_t> bkt_off((size_t)nt + 1, 0);
    for (int32_t t = 0; t < nt; t++) bkt_off[(size_t)t + 1] = bkt_off[(size_t)t] + (int64_t)bk[(size_t)t].size();
    std::vector<uint2> bkt((size_t)bkt_off[(size_t)nt]);
    parallel_for((size_t)nt, 16, [&](size_t t) { std::copy(bk[t].begin(), bk[t].end(), bkt.begin() + bkt_off[t]); });
    // ---- ranges of the index build: ~T stream ops each, cut at read starts and contig starts
    // 32 768 ranges, of at most 65 536 ops: cfg2 index 0.602 -> 0.531 ms, cfg3 2.30 -> 2.19 ms
    // against 131 072 ranges (profiles/r05_J; fewer, longer ranges cross fewer range-boundary
    // slots), while cfg5's 9 G ops keep ~137 K ranges (the stage's 96 events a range).
    constexpr uint64_t IX_TMAX = 65536;
    const uint64_t T = std::min<uint64_t>(std::max<uint64_t>(nstream / c->ix_ranges, 2048), IX_TMAX);
    std::vector<std::vector<uint64_t>> pt((size_t)nt);
    parallel_for((size_t)nt, 16, [&](size_t t) {
        for (int64_t r = tid_off[t], r1 = tid_off[t + 1]; r < r1;) {
            pt[t].push_back((uint64_t)r);
            const uint64_t s0 = soff[r];
            const int64_t rs = r;   // (at most IX_RCAP reads: the single-pass walk stages their offsets)
            for (r++; r < r1 && soff[r] - s0 < T && r - rs < (int64_t)IX_RCAP; r++) {}
        }
    });
    std::vector<uint64_t> part;
    for (int32_t t = 0; t < nt; t++) part.insert(part.end(), pt[(size_t)t].begin(), pt[(size_t)t].end());
    part.push_back((uint64_t)nr);
    if (part.size() - 1 > 0xffffffffull) return fail(c, SVT_EINVAL, "pileup: %s", "too many index ranges");
    c->n_ranges = (uint32_t)(part.size() - 1);
    // the lane-per-read index's 64-read groups: each group's ops < 2^27, so that its events fit
    // the 32-bit wave scans and buffer sizes (else the stream walk builds the index)
    c->n_groups = (uint32_t)((nr + WAVE - 1) / WAVE);
    for (int64_t g0 = 0; g0 < nr && c->n_groups; g0 += WAVE)
        if (soff[std::min<int64_t>(g0 + WAVE, nr)] - soff[g0] >= (1ull << 27)) c->n_groups = 0;
    c->load_stats.host_ms = t_pre_ms + ms_since(t_start);

    const clk::time_point t_up = clk::now();
    svt_status s;
    if ((s = upload(c, c->d_pos, pos, (size_t)nr))) return s;
    if ((s = upload(c, c->d_emax, emax.data(), (size_t)nr))) return s;
    if ((s = upload(c, c->d_rec, rec.data(), (size_t)nr))) return s;
    {
        std::vector<uint8_t> clip8((size_t)std::max<int64_t>(nr, 1), 0);
        for (int64_t r = 0; r < nr; r++) clip8[(size_t)r] = (uint8_t)(nc[r] >> 30);
        if ((s = upload(c, c->d_clip8, clip8.data(), clip8.size()))) return s;
    }
    if ((s = upload(c, c->d_off64, soff, nr > 0 ? (size_t)nr + 1 : 0, nr > 0 ? 0 : 1))) return s;
    if ((s = upload(c, c->d_bkt, bkt.data(), bkt.size()))) return s;
    if ((s = upload(c, c->d_bkt_off, bkt_off.data(), bkt_off.size()))) return s;
    if (nt > 0) { if ((s = upload(c, c->d_tid_off, tid_off, (size_t)nt + 1))) return s; }
    else if ((s = upload<int64_t>(c, c->d_tid_off, nullptr, 0, 1))) return s;
    if (stream_d) c->dev_bytes += (nstream + STREAM_PAD) * 4u;
    else if ((s = upload(c, c->d_cigar, stream_h, (size_t)nstream, STREAM_PAD))) return s;
    if ((s = upload(c, c->d_part, part.data(), part.size()))) return s;
    const size_t S = (size_t)nr + 1;
    if ((s = upload<uint64_t>(c, c->d_spoffD, nullptr, 0, S))) return s;
    if ((s = upload<uint64_t>(c, c->d_spoffI, nullptr, 0, S))) return s;
    if ((s = upload<uint2>(c, c->d_cnt, nullptr, 0, std::max<size_t>((size_t)nr, 1)))) return s;
    const size_t NR = std::max<size_t>({(size_t)c->n_ranges, (size_t)c->n_groups, (size_t)1});
    if ((s = upload<IxTot>(c, c->d_agg, nullptr, 0, NR))) return s;
    const size_t NB = (NR + IX_BLK - 1) / IX_BLK;
    if ((s = upload<IxTot>(c, c->d_bsum, nullptr, 0, NB))) return s;   // (zeroed: the first build adds into them)
    if ((s = upload<IxTot>(c, c->d_bpre, nullptr, 0, NB))) return s;
    HIP_TRY(c, hipMemset(c->d_bsum, 0, NB * sizeof(IxTot)));
    c->n_bsum = NB;
    c->bsum_dirty = false;
    if (c->n_ranges > 0x7fffffffu) return fail(c, SVT_EINVAL, "pileup: %s", "too many index ranges");
    if ((s = upload<uint64_t>(c, c->d_tot, nullptr, 0, IX_NTOT))) return s;
    if (!index_lane(c, nops, (uint64_t)nr)) {   // the stream walk's scratch slots
        const size_t RR = std::max<size_t>(c->n_ranges, 1);
        if ((s = upload<uint4>(c, c->d_scr, nullptr, 0, RR * IX_SCAP))) return s;
        if ((s = upload<uint2>(c, c->d_scrh, nullptr, 0, RR * IX_RCAP))) return s;
        if ((s = upload<uint32_t>(c, c->d_ovf, nullptr, 0, RR))) return s;
    }
    c->load_stats.upload_ms = ms_since(t_up);
    c->n_targets = nt;
    c->n_reads = nr;
    c->n_ops = nops;
    if (nr > 0) {
        double ims = 0;
        if ((s = build_index(c, nullptr, true, &ims))) return s;
        c->load_stats.index_ms = ims;
        const uint64_t R = (uint64_t)nr;
        c->load_stats.span_events = c->n_evD + c->n_evI;
        c->load_stats.lead_blocks = 0;   // (no lead chunks since 0.17: refine_end's stops vote as e + 2)
        c->load_stats.slow_reads = 0;    // (no slow reads since 0.17: walks saturate at 2^30)
        // lane per read: census stream + soff + rec (24 B/read), cnt written (8 B/read); emit cnt
        // + soff + rec (32 B/read) + stream, the per-read offsets (16 B/read) written; the events
        // written.  Stream walk (one pass): stream + soff + rec (24 B/read); the staged offsets
        // (8 B/read) and events written to scratch, read back, written to their places (16 B/read
        // of offsets, 3 x 16 B/event).
        if (c->load_stats.index_kind == 1)
            c->load_stats.index_bytes = 8ull * nstream + 65ull * R + 16ull * (c->n_evD + c->n_evI);
        else
            c->load_stats.index_bytes = 4ull * nstream + 56ull * R + 48ull * (c->n_evD + c->n_evI);
        if (c->bk_on) {   // the value buckets, filed from the stream (short reads) or the span lists
            if ((s = bk_load(c, vtop))) return s;
            if (c->bk_ready) {
                uint64_t placed = 0;
                for (int A = 0; A < BA_N; A++) placed += c->bk_events[A];
                c->load_stats.bucket_index = 1;
                c->load_stats.buckets = c->bk_n;
                c->load_stats.bucket_events = placed;
                c->load_stats.bucket_bytes = c->load_stats.index_kind == 1
                    ? 4ull * nstream + 24ull * R + 28ull * placed
                    : 4ull * nstream + 32ull * R + 32ull * (c->n_evD + c->n_evI) + 28ull * placed;
            }
        }
    } else {
        for (auto *pp : {&c->d_spD, &c->d_spI})
            if ((s = upload<uint4>(c, *pp, nullptr, 0, 1))) return s;
    }
    HIP_TRY(c, hipDeviceSynchronize());
    {
        uint32_t ixerr = 0;
        HIP_TRY(c, hipMemcpy(&ixerr, c->d_ctl + 12, 4, hipMemcpyDeviceToHost));
        if (ixerr) {
            HIP_TRY(c, hipMemset(c->d_ctl + 12, 0, 4));
            return fail(c, SVT_EDEVICE, "%s", "device index build: emit overran the census's sizes");
        }
    }
    c->loaded = true;
    return SVT_OK;
}

static svt_status load_1(svt_ctx *c, const svt_pileup_view *p) {
    if (!c || !p) return SVT_EINVAL;
    if (p->n_targets < 0 || (p->n_targets > 0 && !p->tid_off))
        return fail(c, SVT_EINVAL, "pileup: %s", "bad n_targets / tid_off");
    DEV_GUARD(c);
    free_pileup(c);
    using clk = std::chrono::steady_clock;
    const clk::time_point t_start = clk::now();
    c->load_stats = svt_load_stats{};
    const int32_t nt = p->n_targets;
    const int64_t nr = nt ? p->tid_off[nt] : 0;
    if (nt && p->tid_off[0] != 0) return fail(c, SVT_EINVAL, "pileup: %s", "tid_off[0] != 0");
    for (int32_t t = 0; t < nt; t++)
        if (p->tid_off[t + 1] < p->tid_off[t]) return fail(c, SVT_EINVAL, "pileup: %s", "tid_off not monotone");
    if (nr > 0 && (!p->pos || !p->endpos || !p->cig_off || (!p->cigar && p->cig_off[nr] > 0)))
        return fail(c, SVT_EINVAL, "pileup: %s", "missing arrays");
    const uint64_t nops = nr > 0 ? p->cig_off[nr] : 0;
    if (nr > 0 && p->cig_off[0] != 0) return fail(c, SVT_EINVAL, "pileup: %s", "cig_off[0] != 0");
    // per read n_cigar | clip << 30 (clip from the caller, or from the CIGAR words)
    std::vector<uint32_t> nc((size_t)nr);
    std::vector<int64_t> zeros((size_t)std::max(nt, 1), 0);   // reads with n_cigar == 0 per contig
    std::vector<const char *> bad((size_t)std::max(nt, 1), nullptr);
    parallel_for((size_t)nt, 16, [&](size_t t) {
        for (int64_t r = p->tid_off[t], r1 = p->tid_off[t + 1]; r < r1; r++) {
            const uint64_t o0 = p->cig_off[r], o1 = p->cig_off[r + 1];
            if (o1 < o0 || o1 > nops || o1 - o0 > NCIG_MASK) { bad[t] = "bad cig_off"; return; }
            const uint32_t ncig = (uint32_t)(o1 - o0);
            uint32_t clip;
            if (p->clip) clip = p->clip[r] & 3u;
            else clip = ncig ? (((p->cigar[o1 - 1] & 0xfu) == OP_SOFT ? 1u : 0u) |
                                ((p->cigar[o0] & 0xfu) == OP_SOFT ? 2u : 0u)) : 0u;
            zeros[t] += ncig == 0;
            nc[(size_t)r] = ncig | clip << 30;
        }
    });
    for (int32_t t = 0; t < nt; t++)
        if (bad[(size_t)t]) return fail(c, SVT_EINVAL, "pileup: %s", bad[(size_t)t]);
    // ---- the CIGAR stream: the caller's words; a read with n_cigar == 0 gets one 0M word (no
    // advance, never a candidate) so that every read owns a stream op (svt_index.inc)
    int64_t nzero = 0;
    for (int32_t t = 0; t < nt; t++) nzero += zeros[(size_t)t];
    const uint64_t *soff = p->cig_off;
    const uint32_t *strm = p->cigar;
    std::vector<uint64_t> soff2;
    std::vector<uint32_t> strm2;
    if (nzero > 0) {
        soff2.resize((size_t)nr + 1);
        strm2.reserve(nops + (uint64_t)nzero);
        for (int64_t r = 0; r < nr; r++) {
            soff2[(size_t)r] = strm2.size();
            const uint64_t o0 = p->cig_off[r], o1 = p->cig_off[r + 1];
            if (o1 == o0) strm2.push_back(0u);
            else strm2.insert(strm2.end(), p->cigar + o0, p->cigar + o1);
        }
        soff2[(size_t)nr] = strm2.size();
        soff = soff2.data();
        strm = strm2.data();
    }
    const double pre = std::chrono::duration<double, std::milli>(clk::now() - t_start).count();
    svt_status s = load_core(c, nt, p->tid_off, p->pos, p->endpos, nc.data(), soff, strm, nullptr, nops, pre);
    c->load_stats.total_ms = std::chrono::duration<double, std::milli>(clk::now() - t_start).count();
    return s;
}

// svt_open_multi: run fn(ctx_d, lo_d, hi_d) for the contiguous slices [lo_d, hi_d) of n items,
// one per device, concurrently (one host thread per extra device); the first failure's
// status and message are reported on the parent context.
extern "C++" template <typename F>
static svt_status for_devices(svt_ctx *c, size_t n, F fn) {
    const size_t D = 1 + c->subs.size();
    if (D == 1) return fn(c, (size_t)0, n);
    std::vector<svt_ctx *> ctx(D);
    ctx[0] = c;
    for (size_t d = 1; d < D; d++) ctx[d] = c->subs[d - 1];
    std::vector<svt_status> st(D, SVT_OK);
    const size_t per = (n + D - 1) / D;
    std::vector<std::thread> th;
    for (size_t d = 1; d < D; d++)
        th.emplace_back([&, d] { st[d] = fn(ctx[d], std::min(n, d * per), std::min(n, (d + 1) * per)); });
    st[0] = fn(c, 0, std::min(n, per));
    for (auto &t : th) t.join();
    for (size_t d = 0; d < D; d++)
        if (st[d] != SVT_OK) {
            if (d) snprintf(c->err, sizeof c->err, "device %d: %s", ctx[d]->device, ctx[d]->err);
            return st[d];
        }
    return SVT_OK;
}

svt_status svt_load_pileup(svt_ctx *c, const svt_pileup_view *p) {
    if (!c || !p) return SVT_EINVAL;
    if (c->subs.empty()) return load_1(c, p);
    // every device gets the whole pileup (n = device count: one "item" per device)
    const size_t D = 1 + c->subs.size();
    return for_devices(c, D, [&](svt_ctx *x, size_t lo, size_t hi) { return lo < hi ? load_1(x, p) : SVT_OK; });
}

svt_status svt_reindex(svt_ctx *c, void *stream) {
    if (!c) return SVT_EINVAL;
    if (!c->loaded) return fail(c, SVT_ESTATE, "%s", "svt_load_pileup not called");
    DEV_GUARD(c);
    if (c->n_reads == 0) return SVT_OK;
    const hipStream_t st = (hipStream_t)stream;
    svt_status s = order_on(c, st);   // after every launch already issued (they read the index)
    if (s) return s;
    if (!c->bk_ready) return build_index(c, st, false, nullptr);
    // the value buckets: short reads filed straight from the CIGAR stream; long reads from the
    // span lists, rebuilt first.  A captured build files through its own cursors (zeroed by the
    // graph), a direct one through the epoch cursors (svt_bucket_build.inc).
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (st) HIP_TRY(c, hipStreamIsCapturing(st, &cap));
    const bool captured = cap == hipStreamCaptureStatusActive;
    if (!index_lane(c, c->n_ops, (uint64_t)c->n_reads)) {   // long reads: the stream walk stages the events
        const IxArgs a = ix_args(c);
        hipLaunchKernelGGL(index_kernel, dim3((unsigned)((c->n_ranges + IX_WPB - 1) / IX_WPB)), dim3(64 * IX_WPB), 0, st, a);
        HIP_TRY(c, hipGetLastError());
        c->bsum_dirty = true;   // (its block sums are not scanned: the next span-list build clears them)
    }
    if (captured)
    {   // (the buffer is allocated in whole uint4s: upload's size below rounds it up)
        const uint64_t n4 = (BA_N * (c->bk_n + 1) + 3) / 4;
        hipLaunchKernelGGL(bk_zero_kernel, dim3((unsigned)std::min<uint64_t>((n4 + 255) / 256, 4096)), dim3(256), 0, st,
                           reinterpret_cast<uint4 *>(c->d_bkcap), n4);
        HIP_TRY(c, hipGetLastError());
    }
    if ((s = bk_pass(c, st, false, captured))) return s;
    if (!captured) c->bk_builds++;
    return SVT_OK;
}

svt_status svt_last_load_stats(const svt_ctx *c, svt_load_stats *out) {
    if (!c || !out) return SVT_EINVAL;
    *out = c->load_stats;
    return SVT_OK;
}

static svt_status refine_device_any(svt_ctx *c, const svt_locus *d_loci, size_t n, svt_result *d_out,
                                    svt_record *d_rec, const uint32_t *d_index, uint32_t index_base, void *stream) {
    if (!c) return SVT_EINVAL;
    if (!c->loaded) return fail(c, SVT_ESTATE, "%s", "svt_load_pileup not called");
    if (n && (!d_loci || (!d_out && !d_rec))) return fail(c, SVT_EINVAL, "%s", "null loci/out");
    DEV_GUARD(c);
    return launch(c, d_loci, d_out, n, (hipStream_t)stream, false, d_rec, d_index, index_base);
}

svt_status svt_refine_device(svt_ctx *c, const svt_locus *d_loci, size_t n, svt_result *d_out, void *stream) {
    return refine_device_any(c, d_loci, n, d_out, nullptr, nullptr, 0, stream);
}

svt_status svt_refine_device_records(svt_ctx *c, const svt_locus *d_loci, size_t n, const uint32_t *d_index,
                                     uint32_t index_base, svt_record *d_rec, void *stream) {
    if (c && n && !d_rec) return fail(c, SVT_EINVAL, "%s", "null records");
    return refine_device_any(c, d_loci, n, nullptr, d_rec, d_index, index_base, stream);
}

svt_status svt_sync(svt_ctx *c, void *stream) {
    if (!c) return SVT_EINVAL;
    DEV_GUARD(c);
    HIP_TRY(c, hipStreamSynchronize((hipStream_t)stream));
    if (c->have_last && c->last_stream != (hipStream_t)stream) HIP_TRY(c, hipStreamSynchronize(c->last_stream));
    int32_t st2[2] = {0, 0};
    HIP_TRY(c, hipMemcpy(st2, c->d_ctl + 8, 8, hipMemcpyDeviceToHost));
    int32_t status = st2[0];
    if (st2[1]) {   // the index build's guard fired: census and emit disagreed (an engine bug)
        HIP_TRY(c, hipMemset(c->d_ctl + 12, 0, 4));
        return fail(c, SVT_EDEVICE, "%s",
                    st2[1] == 2   ? "device index build: a look-back never ended (results invalid)"
                    : st2[1] == 3 ? "device index build: an event outside its value bucket's extent (results invalid)"
                                  : "device index build: emit overran the census's sizes (results invalid)");
    }
#if SVT_DIAG == 9
    fprintf(stderr, "[diag] wave-wide (phase 3) windows: %d\n", status >> 8);
    HIP_TRY(c, hipMemset(c->d_ctl + 8, 0, 4));
    status &= 1;
#endif
    if (status & 1) {
        HIP_TRY(c, hipMemset(c->d_ctl + 8, 0, 4));   // sticky until reported
        const svt_status g = grow_pool(c);            // a re-run of the batch now fits
        if (g) return g;
        return fail(c, SVT_EOVERFLOW, "%s", "candidate spill pool exhausted (pool grown; re-run the batch)");
    }
    return SVT_OK;
}

// One synchronous launch over host loci on one device (count: the work-counting kernel);
// a launch whose spilled windows outgrew the pool is re-run once the pool has grown.
static svt_status run_batch_1(svt_ctx *c, const svt_locus *loci, size_t n, svt_result *out, svt_work *w) {
    if (n == 0) return SVT_OK;
    DEV_GUARD(c);
    svt_status s = ensure_batch(c, n);
    if (s) return s;
    HIP_TRY(c, hipMemcpy(c->d_loci, loci, n * sizeof(svt_locus), hipMemcpyHostToDevice));
    for (int attempt = 0;; attempt++) {
        s = launch(c, c->d_loci, c->d_out, n, nullptr, w != nullptr);
        if (s) return s;
        s = svt_sync(c, nullptr);
        if (s != SVT_EOVERFLOW || attempt == 3) break;
    }
    if (s) return s;
    if (out) HIP_TRY(c, hipMemcpy(out, c->d_out, n * sizeof(svt_result), hipMemcpyDeviceToHost));
    if (w) {
        unsigned long long k[W_N];
        HIP_TRY(c, hipMemcpy(k, c->d_ctl + 16, sizeof k, hipMemcpyDeviceToHost));
        w->windows = k[W_WINDOWS]; w->reads = k[W_READS]; w->ops_walked = k[W_OPS]; w->candidates = k[W_CANDS];
        w->spilled_windows = k[W_SPILLED]; w->queries = k[W_QUERIES]; w->probe_entries = k[W_PROBE];
        w->range_reads = k[W_RANGE]; w->list_reads = k[W_LREADS]; w->list_entries = k[W_LENTRIES];
        w->stop_searches = k[W_STOPS]; w->stop_chunk_words = k[W_STOPCH];
        w->span_bounds = k[W_SQUERIES]; w->span_events = k[W_SPAN];
        // algorithmic bytes of the span walk (DESIGN.md "Roofline"): locus in + result out, two
        // bucket words per search pair, the search entries, the two span bounds of a query and
        // its 16-B events, per stop search the chunk words scanned, the word before the break
        // chunk and its 8 CIGAR words
        w->bucket_queries = k[W_BQ];
        w->bucket_events = k[W_BEV];
        w->event_bytes = 24ull * n + 32ull * w->queries + 4ull * w->probe_entries + 36ull * w->stop_searches +
                         4ull * w->stop_chunk_words + 16ull * w->span_bounds + 16ull * w->span_events;
        // the value buckets (svt_bucket.inc): locus in + result out, per window two bucket offsets
        // and one prefix-max key, the 16-B events of its band's buckets and of the walks for ABOVE
        // (windows the buckets do not take -- none at the default parameters -- are not priced)
        if (c->bk_ready) w->event_bytes = 24ull * n + 12ull * w->bucket_queries + 16ull * w->bucket_events;
    }
    return SVT_OK;
}

svt_status svt_refine_batch(svt_ctx *c, const svt_locus *loci, size_t n, svt_result *out) {
    if (!c) return SVT_EINVAL;
    if (!c->loaded) return fail(c, SVT_ESTATE, "%s", "svt_load_pileup not called");
    if (n == 0) return SVT_OK;
    if (!loci || !out) return fail(c, SVT_EINVAL, "%s", "null loci/out");
    return for_devices(c, n, [&](svt_ctx *x, size_t lo, size_t hi) {
        return run_batch_1(x, loci + lo, hi - lo, out + lo, nullptr);
    });
}

svt_status svt_count_work(svt_ctx *c, const svt_locus *loci, size_t n, svt_work *out) {
    if (!c || !out) return SVT_EINVAL;
    if (!c->loaded) return fail(c, SVT_ESTATE, "%s", "svt_load_pileup not called");
    memset(out, 0, sizeof(*out));
    if (n == 0) return SVT_OK;
    if (!loci) return fail(c, SVT_EINVAL, "%s", "null loci");
    std::vector<svt_work> part(1 + c->subs.size());
    std::vector<svt_ctx *> who(part.size(), nullptr);
    const svt_status s = for_devices(c, n, [&](svt_ctx *x, size_t lo, size_t hi) {
        const size_t d = x == c ? 0 : (size_t)(std::find(c->subs.begin(), c->subs.end(), x) - c->subs.begin()) + 1;
        memset(&part[d], 0, sizeof(svt_work));
        return run_batch_1(x, loci + lo, hi - lo, nullptr, &part[d]);
    });
    if (s) return s;
    uint64_t *o = reinterpret_cast<uint64_t *>(out);
    for (const svt_work &p : part) {
        const uint64_t *q = reinterpret_cast<const uint64_t *>(&p);
        for (size_t i = 0; i < sizeof(svt_work) / 8; i++) o[i] += q[i];
    }
    return SVT_OK;
}

uint64_t svt_sw_subwindows(const svt_sw_query *q, int32_t window_size) {
    if (!q || window_size < 1 || q->end <= q->start) return 0;
    return ((uint64_t)(q->end - q->start) + (uint64_t)window_size - 1) / (uint64_t)window_size;
}

static svt_status sw_1(svt_ctx *c, const svt_sw_query *q, size_t n, int32_t window_size, int32_t slide_size,
                       int32_t *best, svt_sw_window *sub);

svt_status svt_sliding_window_ins(svt_ctx *c, const svt_sw_query *q, size_t n, int32_t window_size,
                                  int32_t slide_size, int32_t *best, svt_sw_window *sub) {
    if (!c) return SVT_EINVAL;
    if (!c->loaded) return fail(c, SVT_ESTATE, "%s", "svt_load_pileup not called");
    if (window_size < 1 || slide_size < 1)
        return fail(c, SVT_EINVAL, "%s", "window_size and slide_size must be >= 1 (the reference loops forever)");
    if (n == 0) return SVT_OK;
    if (!q || !best) return fail(c, SVT_EINVAL, "%s", "null queries/best");
    std::vector<uint64_t> soff(n + 1, 0);   // each query's first sub-window in `sub`
    for (size_t i = 0; i < n; i++) soff[i + 1] = soff[i] + svt_sw_subwindows(q + i, window_size);
    return for_devices(c, n, [&](svt_ctx *x, size_t lo, size_t hi) {
        return sw_1(x, q + lo, hi - lo, window_size, slide_size, best + lo, sub ? sub + soff[lo] : nullptr);
    });
}

static svt_status sw_1(svt_ctx *c, const svt_sw_query *q, size_t n, int32_t window_size, int32_t slide_size,
                       int32_t *best, svt_sw_window *sub) {
    if (n == 0) return SVT_OK;
    if (!c->loaded) return fail(c, SVT_ESTATE, "%s", "svt_load_pileup not called");
    std::vector<uint64_t> off(n + 1, 0);
    for (size_t i = 0; i < n; i++) {
        if ((uint64_t)q[i].end + (uint64_t)window_size > 0x100000000ull)
            return fail(c, SVT_EINVAL, "%s", "end + window_size > 2^32 (sub_start wraps, sliding_window.c:12)");
        off[i + 1] = off[i] + svt_sw_subwindows(q + i, window_size);
    }
    const uint64_t ns = off[n];
    if (ns > 0x3fffffffull) return fail(c, SVT_EINVAL, "%s", "more than 2^30-1 sub-windows in one call");
    std::vector<uint4> subs((size_t)ns);
    for (size_t i = 0; i < n; i++) {
        uint64_t k = off[i];
        for (uint32_t ss = q[i].start; ss < q[i].end; ss += (uint32_t)window_size, k++) {   // :12-15
            uint32_t se = ss + (uint32_t)window_size;
            subs[(size_t)k] = make_uint4((uint32_t)q[i].chrom, ss, se > q[i].end ? q[i].end : se, 0u);
        }
    }
    DEV_GUARD(c);
    svt_status so = order_on(c, nullptr);
    if (so) return so;
    uint4 *d_sub = nullptr;
    int2 *d_res = nullptr;
    uint64_t *d_off = nullptr;
    int32_t *d_best = nullptr;
    svt_status s = SVT_OK;
    auto cleanup = [&]() { hfree(d_sub); hfree(d_res); hfree(d_off); hfree(d_best); };
    auto chk = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && s == SVT_OK) s = fail(c, SVT_EDEVICE, what, hipGetErrorString(e));
        return s == SVT_OK;
    };
    if (chk(hipMalloc(&d_sub, std::max<size_t>(1, (size_t)ns) * sizeof(uint4)), "hipMalloc: %s") &&
        chk(hipMalloc(&d_res, std::max<size_t>(1, (size_t)ns) * sizeof(int2)), "hipMalloc: %s") &&
        chk(hipMalloc(&d_off, (n + 1) * sizeof(uint64_t)), "hipMalloc: %s") &&
        chk(hipMalloc(&d_best, n * sizeof(int32_t)), "hipMalloc: %s") &&
        (ns == 0 || chk(hipMemcpy(d_sub, subs.data(), (size_t)ns * sizeof(uint4), hipMemcpyHostToDevice), "H2D: %s")) &&
        chk(hipMemcpy(d_off, off.data(), (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice), "H2D: %s") &&
        chk(hipMemsetAsync(c->d_ctl, 0, CTL_BYTES, nullptr), "hipMemset: %s")) {
        if (ns) {
            KArgs a = make_args(c, nullptr, nullptr, (uint32_t)ns, false);
            a.prm.sw_window = window_size;
            a.prm.sw_slide = slide_size;
            a.sw_sub = d_sub;
            a.sw_out = d_res;
            const dim3 grid((unsigned)((ns + WPB - 1) / WPB)), block(64 * WPB);
            hipLaunchKernelGGL(sw_kernel<G_SPAN>, grid, block, 0, nullptr, a);
            chk(hipGetLastError(), "sw_kernel: %s");
        }
        if (s == SVT_OK) {
            hipLaunchKernelGGL(sw_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, nullptr, d_res,
                               d_off, (uint32_t)n, d_best);
            chk(hipGetLastError(), "sw_reduce_kernel: %s");
        }
        if (s == SVT_OK) s = svt_sync(c, nullptr);
        if (s == SVT_OK) chk(hipMemcpy(best, d_best, n * sizeof(int32_t), hipMemcpyDeviceToHost), "D2H: %s");
        if (s == SVT_OK && sub && ns)
            chk(hipMemcpy(sub, d_res, (size_t)ns * sizeof(int2), hipMemcpyDeviceToHost), "D2H: %s");
    }
    cleanup();
    return s;
}

// ---- allele-consensus mode (POA; no reference behaviour, see svt_poa.inc)
void svt_poa_default_params(svt_poa_params *p) {
    if (p) *p = svt_poa_params{2, 4, 4, 2, 10, 10, 32, 4000, 32768, 20, 64};
}

uint64_t svt_pileup_ins_count(const svt_ctx *c) { return c ? c->n_ins : 0; }

svt_status svt_load_insseq(svt_ctx *c, const svt_insseq_view *v) {
    if (!c || !v) return SVT_EINVAL;
    if (!c->loaded) return fail(c, SVT_ESTATE, "%s", "svt_load_pileup not called");
    if (v->n_ins != c->n_ins) return fail(c, SVT_EINVAL, "insseq: %s", "n_ins differs from the pileup's I >= 50 op count");
    if (v->n_ins >= (1ull << 31)) return fail(c, SVT_EINVAL, "insseq: %s", ">= 2^31 sequences");
    if (v->n_ins && (!v->off || !v->bases)) return fail(c, SVT_EINVAL, "insseq: %s", "missing arrays");
    if (v->n_ins && v->off[0] != 0) return fail(c, SVT_EINVAL, "insseq: %s", "off[0] != 0");
    for (uint64_t k = 0; k < v->n_ins; k++)
        if (v->off[k + 1] < v->off[k]) return fail(c, SVT_EINVAL, "insseq: %s", "off not monotone");
    DEV_GUARD(c);
    hfree(c->d_ins_off);
    hfree(c->d_ins_bases);
    c->insseq_loaded = false;
    const uint64_t nb = v->n_ins ? v->off[v->n_ins] : 0;
    svt_status s;
    if (v->n_ins) { if ((s = upload(c, c->d_ins_off, v->off, (size_t)v->n_ins + 1))) return s; }
    else if ((s = upload<uint64_t>(c, c->d_ins_off, nullptr, 0, 1))) return s;
    if (nb) { if ((s = upload(c, c->d_ins_bases, v->bases, (size_t)nb))) return s; }
    else if ((s = upload<uint8_t>(c, c->d_ins_bases, nullptr, 0, 1))) return s;
    c->insseq_loaded = true;
    return SVT_OK;
}

svt_status svt_poa_consensus(svt_ctx *c, const svt_poa_params *p, const svt_locus *loci, const svt_result *refined,
                             size_t n, int32_t cap, uint8_t *bases, svt_poa_result *res) {
    if (!c || !p) return SVT_EINVAL;
    if (!c->loaded) return fail(c, SVT_ESTATE, "%s", "svt_load_pileup not called");
    if (!c->insseq_loaded) return fail(c, SVT_ESTATE, "%s", "svt_load_insseq not called");
    if (n == 0) return SVT_OK;
    if (!loci || !refined || !res || cap < 0 || (cap > 0 && !bases)) return fail(c, SVT_EINVAL, "%s", "null arrays / cap");
    if (n > 0x3fffffffull) return fail(c, SVT_EINVAL, "%s", "batch too large");
    const int64_t w_max = (int64_t)p->band_b + (int64_t)p->band_f_permille * p->max_len / 1000;
    if (p->match < 0 || p->mismatch < 0 || p->gap_open < 0 || p->gap_ext < 0 || p->band_b < 1 || p->band_f_permille < 0 ||
        p->max_seqs < 1 || p->max_seqs > POA_PIN || p->max_len < 1 || p->max_len > POA_SEQ_MAX || w_max > 63 ||
        p->max_nodes < p->max_len || p->max_nodes > 65000 || p->support_radius < 0 || p->max_support < 1 ||
        p->match > 1000 || p->mismatch > 1000 || p->gap_open > 1000 || p->gap_ext > 1000)
        return fail(c, SVT_EINVAL, "%s", "poa params out of range");
    DEV_GUARD(c);
    return poa_run(c, p, loci, refined, n, cap, bases, res);
}

uint64_t svt_pileup_device_bytes(const svt_ctx *c) { return c ? c->dev_bytes : 0; }

uint64_t svt_poa_deferred(const svt_ctx *c) { return c ? c->poa_deferred : 0; }

svt_status svt_bgzf_inflate_device(svt_ctx *c, const uint8_t *d_comp, const svt_bgzf_block *d_blocks, size_t n,
                                   uint8_t *d_out, void *stream) {
    if (!c) return SVT_EINVAL;
    if (n == 0) return SVT_OK;
    if (!d_comp || !d_blocks || !d_out) return fail(c, SVT_EINVAL, "%s", "null buffer");
    if (n > 0xfffffffeull) return fail(c, SVT_EINVAL, "%s", "more than 2^32 - 2 blocks in one call");
    DEV_GUARD(c);
    const hipStream_t st = (hipStream_t)stream;
    const unsigned grid = (unsigned)std::min<size_t>(n, (size_t)INF_GRID);
    if (!c->d_inferr) HIP_TRY(c, hipMalloc(&c->d_inferr, sizeof(uint32_t)));
    // the scratch slots and the error word are per context: calls on different streams run in
    // submission order (like every other launch of the context)
    if (svt_status s = order_on(c, st)) return s;
    HIP_TRY(c, hipMemsetAsync(c->d_inferr, 0xff, sizeof(uint32_t), st));
    hipLaunchKernelGGL(inflate_kernel, dim3(grid), dim3(WAVE), 0, st, d_comp, d_blocks, 0u, (uint32_t)n, d_out, c->d_inferr);
    HIP_TRY(c, hipGetLastError());
    return SVT_OK;
}

svt_status svt_bgzf_inflate_status(svt_ctx *c, void *stream, uint32_t *bad_block) {
    if (!c || !bad_block) return SVT_EINVAL;
    *bad_block = 0xffffffffu;
    if (!c->d_inferr) return SVT_OK;
    DEV_GUARD(c);
    // the error word belongs to the context's last inflate: order after it, whatever its stream
    const hipStream_t st = (hipStream_t)stream;
    if (svt_status s = order_on(c, st)) return s;
    HIP_TRY(c, hipMemcpyAsync(bad_block, c->d_inferr, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIP_TRY(c, hipStreamSynchronize(st));
    if (*bad_block != 0xffffffffu) {
        char m[64];
        snprintf(m, sizeof m, "%u", *bad_block);
        return fail(c, SVT_EINVAL, "corrupt BGZF block %s (does not inflate to its ISIZE)", m);
    }
    return SVT_OK;
}

svt_status svt_bgzf_inflate(svt_ctx *c, const uint8_t *comp, size_t comp_bytes, const svt_bgzf_block *blocks, size_t n,
                            uint8_t *out, size_t out_bytes) {
    if (!c) return SVT_EINVAL;
    if (n == 0) return SVT_OK;
    if (!comp || !blocks || !out) return fail(c, SVT_EINVAL, "%s", "null buffer");
    for (size_t i = 0; i < n; i++) {   // every block inside its buffers (the kernel trusts the table)
        const svt_bgzf_block &k = blocks[i];
        if (k.clen > 65536u || k.ulen > 65536u || k.coff > comp_bytes || k.clen > comp_bytes - k.coff ||
            k.uoff > out_bytes || k.ulen > out_bytes - k.uoff)
            return fail(c, SVT_EINVAL, "%s", "BGZF block outside its buffers (or over 64 KiB)");
    }
    DEV_GUARD(c);
    svt_status s = order_on(c, nullptr);
    if (s) return s;
    auto grow = [&](auto *&p, size_t &cap, size_t bytes) -> svt_status {
        if (bytes <= cap) return SVT_OK;
        hfree(p);
        cap = 0;
        HIP_TRY(c, hipMalloc(&p, bytes));
        cap = bytes;
        return SVT_OK;
    };
    if ((s = grow(c->d_infc, c->infc_cap, comp_bytes + 64)) || (s = grow(c->d_info, c->info_cap, std::max<size_t>(out_bytes, 1))) ||
        (s = grow(c->d_infb, c->infb_cap, n * sizeof(svt_bgzf_block))))
        return s;
    HIP_TRY(c, hipMemcpy(c->d_infc, comp, comp_bytes, hipMemcpyHostToDevice));
    HIP_TRY(c, hipMemcpy(c->d_infb, blocks, n * sizeof(svt_bgzf_block), hipMemcpyHostToDevice));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    HIP_TRY(c, hipEventCreate(&e0));
    HIP_TRY(c, hipEventCreate(&e1));
    (void)hipEventRecord(e0, nullptr);
    s = svt_bgzf_inflate_device(c, c->d_infc, c->d_infb, n, c->d_info, nullptr);
    (void)hipEventRecord(e1, nullptr);
    uint32_t bad = 0;
    if (s == SVT_OK) s = svt_bgzf_inflate_status(c, nullptr, &bad);
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e0, e1) == hipSuccess) c->inf_ms = ms;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (s) return s;
    HIP_TRY(c, hipMemcpy(out, c->d_info, out_bytes, hipMemcpyDeviceToHost));
    return SVT_OK;
}

double svt_bgzf_last_inflate_ms(const svt_ctx *c) { return c ? c->inf_ms : 0.0; }

void *svt_host_alloc(svt_ctx *c, size_t bytes) {
    if (!c) return nullptr;
    DevGuard dg(c->device);
    void *p = nullptr;
    return hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) == hipSuccess ? p : nullptr;
}

void svt_host_free(svt_ctx *c, void *p) {
    if (!c || !p) return;
    DevGuard dg(c->device);
    (void)hipHostFree(p);
}

// ---- BAM records decoded on the device (svt_bam.inc)
}  // extern "C"

// svt_bam_dec_feed is pipelined one batch deep: a call copies its batch's compressed bytes to the
// device (a copy stream, into one of two input buffers) while the previous batch still inflates,
// then decodes the previous batch (whose carried tail fixes where this batch's bytes go) and
// launches this batch's inflate; the next call or svt_bam_dec_load decodes it.  (Copying a batch in
// parts beside its own inflate measured slower: every part's launch waits for its slowest block,
// profiles/r05_I.)
struct svt_bam_dec {
    svt_ctx *c = nullptr;
    int32_t n_ref = 0;
    hipStream_t st = nullptr;
    hipStream_t cst = nullptr;                // the copy stream
    hipEvent_t cev = nullptr;                 // the latest batch's bytes are on the device
    uint8_t *d_comp[2] = {nullptr, nullptr};  // compressed batches (alternating)
    size_t comp_cap[2] = {0, 0};
    svt_bgzf_block *d_blk[2] = {nullptr, nullptr};
    size_t blk_cap[2] = {0, 0};
    int ib = 0;                               // the next batch's input buffer
    uint32_t *d_err = nullptr;                // the inflate's first bad block (this decoder's own word)
    bool pend = false;                        // a batch inflated (or inflating) but not yet decoded
    size_t pend_n = 0;
    uint64_t pend_u = 0, pend_r0 = 0;
    uint8_t *d_buf[2] = {nullptr, nullptr};   // inflated batches: [carried tail | this batch]
    size_t buf_cap[2] = {0, 0};
    int cur = 0;
    uint64_t tail = 0;                        // bytes of the incomplete record at the front of d_buf[cur]
    bool first = true;
    BdChunk *d_ch = nullptr;
    uint32_t *d_base = nullptr;
    size_t ch_cap = 0, base_cap = 0;
    BdRec *d_rec = nullptr;
    BdTot *d_pre = nullptr;
    size_t rec_cap = 0, pre_cap = 0;
    BdCheck *d_chk = nullptr;
    void *d_tmp = nullptr;
    size_t tmp_cap = 0;
    BdCols cols{};
    uint64_t col_cap = 0, word_cap = 0;       // capacities of the columns (reads) and the stream (words)
    uint64_t nkept = 0, nwords = 0;
    svt_bam_dec_stats stats{};
};

namespace {
template <typename T>
svt_status bd_grow(svt_ctx *c, T *&p, size_t &cap, size_t need, size_t keep = 0) {   // device, keeping `keep` elements
    if (need <= cap) return SVT_OK;
    const size_t nc = std::max(need, cap + cap / 2);
    T *q = nullptr;
    if (hipMalloc(&q, nc * sizeof(T)) != hipSuccess) return fail(c, SVT_ENOMEM, "%s", "device memory for the BAM decode");
    if (keep && p) HIP_TRY(c, hipMemcpy(q, p, keep * sizeof(T), hipMemcpyDeviceToDevice));
    hfree(p);
    p = q;
    cap = nc;
    return SVT_OK;
}
}  // namespace

extern "C" {

svt_status svt_bam_dec_open(svt_ctx *c, int32_t n_targets, svt_bam_dec **out) {
    if (!c || !out || n_targets < 0) return SVT_EINVAL;
    *out = nullptr;
    DEV_GUARD(c);
    svt_bam_dec *d = new (std::nothrow) svt_bam_dec();
    if (!d) return fail(c, SVT_ENOMEM, "%s", "host memory");
    d->c = c;
    d->n_ref = n_targets;
    const bool ok = hipStreamCreateWithFlags(&d->st, hipStreamNonBlocking) == hipSuccess &&
                    hipStreamCreateWithFlags(&d->cst, hipStreamNonBlocking) == hipSuccess &&
                    hipEventCreateWithFlags(&d->cev, hipEventDisableTiming) == hipSuccess &&
                    hipMalloc(&d->d_chk, sizeof(BdCheck)) == hipSuccess && hipMalloc(&d->d_err, sizeof(uint32_t)) == hipSuccess;
    if (!ok) {
        svt_bam_dec_close(d);
        return fail(c, SVT_EDEVICE, "%s", "BAM decode: stream / buffers");
    }
    *out = d;
    return SVT_OK;
}

namespace {
// The pending batch's records: it was inflated into d_buf[cur] after the carried tail (its
// kernels run on d->st, so the decode's launches wait for them).  The incomplete last record
// moves to the front of the other buffer.
svt_status bd_decode(svt_bam_dec *d) {
    svt_ctx *c = d->c;
    svt_status s;
    d->pend = false;
    uint8_t *buf = d->d_buf[d->cur];
    const uint64_t N = d->tail + d->pend_u, r0 = d->pend_r0;
    const uint64_t span = N - r0;
    const uint32_t nch = (uint32_t)((span + BD_CHUNK - 1) / BD_CHUNK);
    BdCheck chk{1u, 0u, 0ull, N, 0u, 0u, 0ull};
    if (nch) {
        if ((s = bd_grow(c, d->d_ch, d->ch_cap, nch)) || (s = bd_grow(c, d->d_base, d->base_cap, nch))) return s;
        hipLaunchKernelGGL(bd_chunk_kernel, dim3(nch), dim3(WAVE), 0, d->st, buf, r0, N, nch, d->n_ref, d->d_ch);
        hipLaunchKernelGGL(bd_check_kernel, dim3(1), dim3(WAVE), 0, d->st, buf, d->d_ch, nch, r0, N, d->d_chk);
        HIP_TRY(c, hipGetLastError());
        uint32_t ierr = 0xffffffffu;
        HIP_TRY(c, hipMemcpyAsync(&chk, d->d_chk, sizeof chk, hipMemcpyDeviceToHost, d->st));
        HIP_TRY(c, hipMemcpyAsync(&ierr, d->d_err, sizeof ierr, hipMemcpyDeviceToHost, d->st));
        HIP_TRY(c, hipStreamSynchronize(d->st));
        if (d->pend_n && ierr != 0xffffffffu) {
            char m[64];
            snprintf(m, sizeof m, "%u", ierr);
            return fail(c, SVT_EINVAL, "corrupt BGZF block %s of the batch (does not inflate to its ISIZE)", m);
        }
        if (!chk.ok) {   // a wrong guess: the exact chain, hop by hop from the first wrong chunk on
            d->stats.rechained++;
            d->stats.rechained_chunks += nch - chk.kfail;
            hipLaunchKernelGGL(bd_chain_kernel, dim3(1), dim3(WAVE), 0, d->st, buf, r0, N, nch, chk.kfail, chk.efail,
                               d->d_ch);
            hipLaunchKernelGGL(bd_check_kernel, dim3(1), dim3(WAVE), 0, d->st, buf, d->d_ch, nch, r0, N, d->d_chk);
            HIP_TRY(c, hipGetLastError());
            HIP_TRY(c, hipMemcpyAsync(&chk, d->d_chk, sizeof chk, hipMemcpyDeviceToHost, d->st));
            HIP_TRY(c, hipStreamSynchronize(d->st));
            if (!chk.ok) return fail(c, SVT_EDEVICE, "%s", "BAM decode: the exact record chain failed its own check");
        }
        if (chk.bad) return fail(c, SVT_EINVAL, "%s", "corrupt BAM record (block_size < 32)");
    }
    if (chk.nrec) {
        const uint64_t nrec = chk.nrec;
        if (nrec >= 0xffffffffull) return fail(c, SVT_EINVAL, "%s", "BAM decode: more than 2^32 records in one batch");
        if ((s = bd_grow(c, d->d_rec, d->rec_cap, nrec)) || (s = bd_grow(c, d->d_pre, d->pre_cap, nrec))) return s;
        // the chunks' record counts -> their first record's index; the records; their kept / word prefixes
        const auto cnt = hipcub::TransformInputIterator<uint32_t, BdCntOf, const BdChunk *>(d->d_ch, BdCntOf());
        const auto tot = hipcub::TransformInputIterator<BdTot, BdTotOf, const BdRec *>(d->d_rec, BdTotOf());
        size_t need1 = 0, need2 = 0;
        HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(nullptr, need1, cnt, d->d_base, (int)chk.nk, d->st));
        HIP_TRY(c, hipcub::DeviceScan::ExclusiveScan(nullptr, need2, tot, d->d_pre, BdTotSum(), BdTot{0, 0, 0, 0, 0},
                                                     (int)nrec, d->st));
        if ((s = bd_grow(c, reinterpret_cast<uint8_t *&>(d->d_tmp), d->tmp_cap, std::max(need1, need2)))) return s;
        size_t t1 = d->tmp_cap, t2 = d->tmp_cap;
        HIP_TRY(c, hipcub::DeviceScan::ExclusiveSum(d->d_tmp, t1, cnt, d->d_base, (int)chk.nk, d->st));
        hipLaunchKernelGGL(bd_rec_kernel, dim3(chk.nk), dim3(WAVE), 0, d->st, buf, d->d_ch, d->d_base, chk.nk, d->n_ref,
                           d->d_rec);
        HIP_TRY(c, hipGetLastError());
        HIP_TRY(c, hipcub::DeviceScan::ExclusiveScan(d->d_tmp, t2, tot, d->d_pre, BdTotSum(), BdTot{0, 0, 0, 0, 0},
                                                     (int)nrec, d->st));
        BdTot last{};
        BdRec lr{};
        HIP_TRY(c, hipMemcpyAsync(&last, d->d_pre + nrec - 1, sizeof last, hipMemcpyDeviceToHost, d->st));
        HIP_TRY(c, hipMemcpyAsync(&lr, d->d_rec + nrec - 1, sizeof lr, hipMemcpyDeviceToHost, d->st));
        HIP_TRY(c, hipStreamSynchronize(d->st));
        const BdTot all = BdTotSum()(last, BdTotOf()(lr));
        if (all.bad) return fail(c, SVT_EINVAL, "%s", "corrupt BAM record");
        // the columns and the stream (STREAM_PAD spare words), grown keeping what they hold
        const uint64_t G = d->nkept + all.keep + 1, W = d->nwords + all.words + STREAM_PAD;
        if (G > d->col_cap) {   // every column to the same capacity
            size_t cc;
            cc = d->col_cap; if ((s = bd_grow(c, d->cols.tid, cc, G, d->nkept))) return s;
            cc = d->col_cap; if ((s = bd_grow(c, d->cols.pos, cc, G, d->nkept))) return s;
            cc = d->col_cap; if ((s = bd_grow(c, d->cols.endpos, cc, G, d->nkept))) return s;
            cc = d->col_cap; if ((s = bd_grow(c, d->cols.nc, cc, G, d->nkept))) return s;
            cc = d->col_cap; if ((s = bd_grow(c, d->cols.soff, cc, G, d->nkept))) return s;
            d->col_cap = cc;
        }
        if ((s = bd_grow(c, d->cols.stream, d->word_cap, W, d->nwords))) return s;
        hipLaunchKernelGGL(bd_copy_kernel, dim3((unsigned)std::min<uint64_t>((nrec + 3) / 4, 16384)), dim3(256), 0, d->st,
                           buf, d->d_rec, d->d_pre, nrec, d->cols, d->nkept, d->nwords);
        HIP_TRY(c, hipGetLastError());
        d->nkept += all.keep;
        d->nwords += all.words;
        d->stats.records += nrec;
        d->stats.reads += all.keep;
        d->stats.cigar_ops += all.ops;
        d->stats.cg_restored += all.cg;
    }
    // the incomplete last record moves to the front of the other buffer
    const uint64_t nt = N - chk.tail;
    int nx = d->cur ^ 1;
    if ((s = bd_grow(c, d->d_buf[nx], d->buf_cap[nx], std::max<uint64_t>(nt, 1) + 64))) return s;
    if (nt) HIP_TRY(c, hipMemcpyAsync(d->d_buf[nx], buf + chk.tail, nt, hipMemcpyDeviceToDevice, d->st));
    HIP_TRY(c, hipStreamSynchronize(d->st));
    d->cur = nx;
    d->tail = nt;
    return SVT_OK;
}
}  // namespace

svt_status svt_bam_dec_feed(svt_bam_dec *d, const uint8_t *comp, size_t comp_bytes, const svt_bgzf_block *blocks,
                            size_t n, uint64_t skip) {
    if (!d) return SVT_EINVAL;
    svt_ctx *c = d->c;
    if (n && (!comp || !blocks)) return fail(c, SVT_EINVAL, "%s", "null buffer");
    if (n > 0xfffffffeull) return fail(c, SVT_EINVAL, "%s", "more than 2^32 - 2 blocks in one call");
    uint64_t U = 0, lo = ~0ull, hi = 0;
    for (size_t i = 0; i < n; i++) {   // every block inside its buffers (the kernel trusts the table)
        const svt_bgzf_block &k = blocks[i];
        if (k.clen > 65536u || k.ulen > 65536u || k.coff > comp_bytes || k.clen > comp_bytes - k.coff)
            return fail(c, SVT_EINVAL, "%s", "BGZF block outside its buffers (or over 64 KiB)");
        U = std::max<uint64_t>(U, k.uoff + k.ulen);
        lo = std::min<uint64_t>(lo, k.coff);
        hi = std::max<uint64_t>(hi, k.coff + k.clen);
    }
    DEV_GUARD(c);
    using clk = std::chrono::steady_clock;
    const clk::time_point t0 = clk::now();
    svt_status s;
    const uint64_t r0 = d->first ? skip : 0;   // (the first batch carries no tail)
    if (r0 > (d->first ? 0 : d->tail) + U) return fail(c, SVT_EINVAL, "%s", "BAM decode: the header runs past the first batch");
    d->first = false;
    // this batch's bytes cross PCIe while the previous batch inflates (its input is the other buffer)
    const int ib = d->ib;
    d->ib ^= 1;
    if ((s = bd_grow(c, d->d_comp[ib], d->comp_cap[ib], comp_bytes + 64)) ||
        (s = bd_grow(c, d->d_blk[ib], d->blk_cap[ib], std::max<size_t>(n, 1))))
        return s;
    // Once this batch's copies are queued, every return waits for them first: the header lets the
    // caller reuse `comp` / `blocks` as soon as the call returns, error returns included.
    struct CopyWait {
        hipStream_t cst = nullptr;
        ~CopyWait() {
            if (cst) (void)hipStreamSynchronize(cst);
        }
    } copy_wait;
    if (n) {
        copy_wait.cst = d->cst;
        HIP_TRY(c, hipMemcpyAsync(d->d_blk[ib], blocks, n * sizeof(svt_bgzf_block), hipMemcpyHostToDevice, d->cst));
        if (hi > lo) HIP_TRY(c, hipMemcpyAsync(d->d_comp[ib] + lo, comp + lo, hi - lo, hipMemcpyHostToDevice, d->cst));
        HIP_TRY(c, hipEventRecord(d->cev, d->cst));
    }
    // the previous batch's records: fixes the carried tail this batch's bytes follow
    if (d->pend && (s = bd_decode(d))) return s;
    const uint64_t T = d->tail, N = T + U;
    if ((s = bd_grow(c, d->d_buf[d->cur], d->buf_cap[d->cur], N + 64, T))) return s;
    if (n) {
        if ((s = order_on(c, d->st))) return s;
        HIP_TRY(c, hipMemsetAsync(d->d_err, 0xff, sizeof(uint32_t), d->st));
        HIP_TRY(c, hipStreamWaitEvent(d->st, d->cev, 0));
        const unsigned grid = (unsigned)std::min<size_t>(n, (size_t)INF_GRID);
        hipLaunchKernelGGL(inflate_kernel, dim3(grid), dim3(WAVE), 0, d->st, d->d_comp[ib], d->d_blk[ib], 0u, (uint32_t)n,
                           d->d_buf[d->cur] + T, d->d_err);
        HIP_TRY(c, hipGetLastError());
        HIP_TRY(c, hipEventSynchronize(d->cev));   // the caller may reuse its buffers
        copy_wait.cst = nullptr;
    }
    d->pend = true;
    d->pend_n = n;
    d->pend_u = U;
    d->pend_r0 = r0;
    d->stats.batches++;
    d->stats.inflated_bytes += U;
    d->stats.feed_ms += std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    return SVT_OK;
}

#if SVT_PHASE_PROF
// diagnostic builds: refine_lane_kernel's phase times and counts since the last call (then cleared)
int svt_diag_phase(unsigned long long *out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ph_prof), sizeof ph_prof) != hipSuccess) return 1;
    const unsigned long long z[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(ph_prof), z, sizeof z) != hipSuccess;
}
#endif

svt_status svt_bam_dec_stats_get(const svt_bam_dec *d, svt_bam_dec_stats *out) {
    if (!d || !out) return SVT_EINVAL;
    *out = d->stats;
    return SVT_OK;
}

svt_status svt_bam_dec_load(svt_bam_dec *d) {
    if (!d) return SVT_EINVAL;
    svt_ctx *c = d->c;
    DEV_GUARD(c);
    using clk = std::chrono::steady_clock;
    if (d->pend) {   // the last batch's records
        const clk::time_point tf = clk::now();
        const svt_status sd = bd_decode(d);
        d->stats.feed_ms += std::chrono::duration<double, std::milli>(clk::now() - tf).count();
        if (sd) return sd;
    }
    if (d->tail) return fail(c, SVT_EINVAL, "%s", "truncated BAM record at end of file");
    const clk::time_point t0 = clk::now();
    free_pileup(c);
    c->load_stats = svt_load_stats{};
    const int32_t nt = d->n_ref;
    const uint64_t n = d->nkept;
    svt_status s;
    // sortedness and the contig boundaries, on the device
    int64_t *d_toff = nullptr;
    uint32_t *d_uns = nullptr;
    HIP_TRY(c, hipMalloc(&d_toff, ((size_t)nt + 1) * sizeof(int64_t)));
    if (hipMalloc(&d_uns, sizeof(uint32_t)) != hipSuccess) { hfree(d_toff); return fail(c, SVT_ENOMEM, "%s", "device"); }
    std::vector<int64_t> toff((size_t)nt + 1, 0);
    uint32_t uns = 0;
    hipError_t e = hipMemsetAsync(d_uns, 0, sizeof(uint32_t), d->st);
    if (e == hipSuccess) e = hipMemsetAsync(d_toff, 0, ((size_t)nt + 1) * sizeof(int64_t), d->st);
    if (e == hipSuccess) {
        const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 256) / 256, 65536));
        hipLaunchKernelGGL(bd_finish_kernel, dim3(g), dim3(256), 0, d->st, d->cols.tid, d->cols.pos, n, nt, d_toff, d_uns);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(toff.data(), d_toff, toff.size() * sizeof(int64_t), hipMemcpyDeviceToHost, d->st);
    if (e == hipSuccess) e = hipMemcpyAsync(&uns, d_uns, sizeof uns, hipMemcpyDeviceToHost, d->st);
    if (e == hipSuccess) e = hipStreamSynchronize(d->st);
    hfree(d_toff);
    hfree(d_uns);
    if (e != hipSuccess) return fail(c, SVT_EDEVICE, "BAM decode finish: %s", hipGetErrorString(e));
    // the per-read columns the host pass reads (pos, endpos, n_cigar | clip, stream offsets)
    std::vector<int32_t> pos(n), endpos(n), tid(uns ? n : 0);
    std::vector<uint32_t> nc(n);
    std::vector<uint64_t> soff(n + 1);
    if (n) {
        HIP_TRY(c, hipMemcpy(pos.data(), d->cols.pos, n * 4, hipMemcpyDeviceToHost));
        HIP_TRY(c, hipMemcpy(endpos.data(), d->cols.endpos, n * 4, hipMemcpyDeviceToHost));
        HIP_TRY(c, hipMemcpy(nc.data(), d->cols.nc, n * 4, hipMemcpyDeviceToHost));
        HIP_TRY(c, hipMemcpy(soff.data(), d->cols.soff, n * 8, hipMemcpyDeviceToHost));
        if (uns) HIP_TRY(c, hipMemcpy(tid.data(), d->cols.tid, n * 4, hipMemcpyDeviceToHost));
    }
    soff[n] = d->nwords;
    const double pre = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    if (uns) {   // not coordinate-sorted: sort on the host (stable, by tid then pos), as the host ingest does
        std::vector<uint32_t> strm(d->nwords);
        if (d->nwords) HIP_TRY(c, hipMemcpy(strm.data(), d->cols.stream, d->nwords * 4, hipMemcpyDeviceToHost));
        std::vector<size_t> idx(n);
        for (size_t i = 0; i < n; i++) idx[i] = i;
        std::stable_sort(idx.begin(), idx.end(), [&](size_t x, size_t y) {
            return tid[x] != tid[y] ? tid[x] < tid[y] : pos[x] < pos[y];
        });
        std::vector<int32_t> p2(n), e2(n);
        std::vector<uint32_t> n2(n), s2;
        std::vector<uint64_t> o2(n + 1);
        s2.reserve(d->nwords);
        std::fill(toff.begin(), toff.end(), 0);
        for (size_t k = 0; k < n; k++) {
            const size_t i = idx[k];
            p2[k] = pos[i]; e2[k] = endpos[i]; n2[k] = nc[i];
            o2[k] = s2.size();
            s2.insert(s2.end(), strm.begin() + (ptrdiff_t)soff[i], strm.begin() + (ptrdiff_t)soff[i + 1]);
            toff[(size_t)tid[i] + 1]++;
        }
        o2[n] = s2.size();
        for (int32_t t = 0; t < nt; t++) toff[(size_t)t + 1] += toff[(size_t)t];
        s = load_core(c, nt, toff.data(), p2.data(), e2.data(), n2.data(), o2.data(), s2.data(), nullptr,
                      d->stats.cigar_ops, pre);
    } else {
        // the stream stays where the decode wrote it (its spare words zeroed): the context adopts it;
        // a BAM without records never allocated one, so it gets just the spare words here
        if ((s = bd_grow(c, d->cols.stream, d->word_cap, d->nwords + STREAM_PAD, d->nwords))) return s;
        HIP_TRY(c, hipMemset(d->cols.stream + d->nwords, 0, STREAM_PAD * 4));
        s = load_core(c, nt, toff.data(), pos.data(), endpos.data(), nc.data(), soff.data(), nullptr, d->cols.stream,
                      d->stats.cigar_ops, pre);
        if (c->d_cigar == d->cols.stream) {
            d->cols.stream = nullptr;
            d->word_cap = 0;
        }
    }
    c->load_stats.total_ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    return s;
}

void svt_bam_dec_close(svt_bam_dec *d) {
    if (!d) return;
    {
        DevGuard dg(d->c->device);
        if (d->st) (void)hipStreamSynchronize(d->st);
        // the context's launch order may point at this stream (svt_bam_dec_feed's order_on): all of
        // its work is done, so nothing later has to wait for it, and it must not be named again
        if (d->c->have_last && d->c->last_stream == d->st) d->c->have_last = false;
        if (d->cst) (void)hipStreamSynchronize(d->cst);
        hfree(d->d_comp[0]); hfree(d->d_comp[1]); hfree(d->d_blk[0]); hfree(d->d_blk[1]); hfree(d->d_err);
        hfree(d->d_buf[0]); hfree(d->d_buf[1]);
        hfree(d->d_ch); hfree(d->d_base); hfree(d->d_rec); hfree(d->d_pre); hfree(d->d_chk); hfree(d->d_tmp);
        hfree(d->cols.tid); hfree(d->cols.pos); hfree(d->cols.endpos); hfree(d->cols.nc); hfree(d->cols.soff);
        hfree(d->cols.stream);
        if (d->cev) (void)hipEventDestroy(d->cev);
        if (d->st) (void)hipStreamDestroy(d->st);
        if (d->cst) (void)hipStreamDestroy(d->cst);
    }
    delete d;
}

void svt_close(svt_ctx *c) {
    if (!c) return;
    for (svt_ctx *d : c->subs) svt_close(d);
    c->subs.clear();
    DevGuard dg(c->device);
    if (c->order_ev) (void)hipEventDestroy(c->order_ev);
    free_pileup(c);
    hfree(c->d_infc); hfree(c->d_info); hfree(c->d_infb); hfree(c->d_inferr);
    hfree(c->d_loci); hfree(c->d_out); hfree(c->d_pool); hfree(c->d_ctl); hfree(c->d_redo); hfree(c->poa_small.d); hfree(c->poa_big.d);
    delete c;
}

}  // extern "C"
