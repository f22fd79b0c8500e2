// svt_engine.hip -- MI355X (gfx950) SV-refinement engine: HIP kernels + the C ABI of
// include/svtrek_gpu.h.
//
// One wavefront (one 64-lane workgroup) per SV locus.  Per query window the wave
//   1. finds the candidate read range with two 64-ary searches over HBM-resident,
//      per-contig pos[] (sorted) and emax[] (prefix max of endpos) arrays   -- A3
//   2. tests 64 reads per step against htslib's overlap rule (16-B records, coalesced)
//   3. walks each yielded read's CIGAR 64 ops per step: one coalesced 256-B load, a DPP
//      inclusive prefix scan of the reference advance gives every op's reference
//      position at once, a ballot finds the first op past the window end (the break of
//      refinement.c:145-148), and ballots compact the breakpoint candidates into LDS -- A4..A6
//   4. bitonic-sorts the candidates in LDS and runs consensus_pos's asymmetric vote with
//      per-element cluster counts computed in parallel (binary search + int64 prefix
//      sums) and the greedy accept done with scalar readlanes                      -- A8..A10
// Windows with more than SVT_LDS_CANDS candidates re-run the same code on a slab taken
// from a device spill pool, so results stay exact.  No floating point anywhere; no MFMA
// (integer scan + vote, HBM/latency bound).
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <new>
#include <vector>

#include "../../include/svtrek_gpu.h"

#define SVT_VERSION "svtrek_amd 0.1.0 (gfx950)"

namespace {

constexpr int WAVE = 64;
constexpr int CAP = SVT_LDS_CANDS;          // LDS candidates per window
constexpr int SV_MIN_LENGTH = 50;           // params.h:33
constexpr uint32_t OP_INS = 1, OP_DEL = 2, OP_SOFT = 4;   // params.h:11-14
constexpr int K_START = 0, K_END = 1, K_INS = 2;          // refine_start / refine_end / refine_ins
constexpr int32_t T_INS = 1, T_DEL = 2;

struct DevPileup {
    const int32_t *pos;      // [n_reads]
    const int32_t *emax;     // [n_reads] prefix max of endpos within the contig
    const uint4 *rec;        // [n_reads] {endpos, n_cig | clip<<30, cig_off lo, cig_off hi}
    const int64_t *tid_off;  // [n_targets+1]
    const uint32_t *cigar;
    int32_t n_targets;
};

struct KParams {
    int32_t wider, median, narrow, range, ci, min_count;
};

struct KArgs {
    DevPileup pile;
    KParams prm;
    const svt_locus *loci;
    svt_result *out;
    uint32_t n;
    int32_t *pool;              // spill slabs (int32 words)
    unsigned long long *pool_head;
    unsigned long long pool_words;
    int32_t *status;            // bit0: spill pool exhausted
    unsigned long long *work;   // svt_work counters (COUNT builds only)
};

// ------------------------------------------------------------------ wave primitives
__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

__device__ __forceinline__ uint64_t ballot(bool p) { return (uint64_t)__ballot(p); }

__device__ __forceinline__ uint32_t rdlane(uint32_t v, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ int32_t rdlane_i(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t rdlane64(uint64_t v, int l) {
    uint32_t lo = rdlane((uint32_t)v, l), hi = rdlane((uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ int32_t uniform_i(int32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Inclusive wave64 prefix sum (mod 2^32) with DPP: row_shr 1/2/4/8 inside each 16-lane
// row, then row_bcast:15 (rows 1,3) and row_bcast:31 (rows 2,3).
__device__ __forceinline__ uint32_t wave_scan_add(uint32_t x) {
    uint32_t v = x;
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
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
__device__ __forceinline__ int64_t wave_partition_point(int64_t l, int64_t h, Pred pred) {
    const int ln = lane_id();
    while (h - l > WAVE) {
        // probe 64 evenly spaced points p_k = l + (k+1)*(h-l)/65, k = 0..63
        int64_t span = h - l;
        int64_t p = l + ((int64_t)(ln + 1) * span) / (WAVE + 1);
        bool t = pred(p);
        uint64_t m = ballot(t);
        // all probes before the first true probe are false
        int k = m ? __builtin_ctzll(m) : WAVE;
        int64_t nl = k == 0 ? l : l + ((int64_t)k * span) / (WAVE + 1) + 1;
        int64_t nh = k == WAVE ? h : l + ((int64_t)(k + 1) * span) / (WAVE + 1) + 1;
        if (nh > h) nh = h;
        l = nl;
        h = nh;
    }
    // final: at most 64 elements
    int64_t p = l + ln;
    bool t = p < h && pred(p);
    uint64_t m = ballot(t);
    return m ? l + __builtin_ctzll(m) : h;
}

// ------------------------------------------------------------------ candidate sink
struct Sink {
    int32_t *buf;   // LDS or a global spill slab
    int32_t cap;
    int32_t n;      // total candidates seen (may exceed cap: then a spill re-run follows)
    __device__ __forceinline__ void push(bool pred, int32_t val) {
        uint64_t m = ballot(pred);
        if (!m) return;
        int ln = lane_id();
        int idx = n + __popcll(m & ((1ull << ln) - 1ull));
        if (pred && idx < cap) buf[idx] = val;
        n += __popcll(m);
    }
};

template <bool COUNT>
struct WinStats {
    unsigned long long reads = 0, ops = 0;
};

// Walk one yielded read's CIGAR (refinement.c:118-159 / :184-221 / :295-318).
template <int KIND, bool COUNT>
__device__ __forceinline__ void walk_read(const uint32_t *__restrict__ cigar, uint64_t off, uint32_t n,
                                          uint32_t rpos, uint32_t clip, uint32_t s, uint32_t e,
                                          Sink &sink, WinStats<COUNT> &st) {
    const int ln = lane_id();
    uint32_t carry = rpos;
    bool broke = false;
    uint32_t stop_rp = 0;
    uint32_t walked = n;
    for (uint32_t cb = 0; cb < n; cb += WAVE) {
        uint32_t i = cb + (uint32_t)ln;
        bool v = i < n;
        uint32_t w = v ? __builtin_nontemporal_load(cigar + off + i) : 0u;
        uint32_t op = w & 0xfu, len = w >> 4;
        uint32_t adv = (op != OP_INS && op != OP_SOFT) ? len : 0u;   // refinement.c:141
        uint32_t after = carry + wave_scan_add(adv);
        uint32_t before = after - adv;
        uint64_t bm = ballot(v && after > e);                         // refinement.c:145
        int fb = bm ? __builtin_ctzll(bm) : WAVE;
        bool in = v && ln <= fb;
        bool hit;
        if (KIND == K_INS) hit = in && op == OP_INS && (uint32_t)SV_MIN_LENGTH <= len;   // :299
        else hit = in && op == OP_DEL && (uint32_t)SV_MIN_LENGTH < len;                 // :124,:190
        int32_t val = KIND == K_END ? (int32_t)(before + len + 1u) : (int32_t)before;   // :198/:136
        sink.push(hit, val);
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

// Region query + walks of one window; returns candidates seen (sink.n).
template <int KIND, bool COUNT>
__device__ int32_t gather_window(const DevPileup &P, int tid, uint32_t s, uint32_t e, Sink &sink,
                                 WinStats<COUNT> &st) {
    // sam_itr_queryi(idx, chrom-1, inter.start-1, inter.end-1), refinement.c:114
    const int64_t beg = (int64_t)(uint32_t)(s - 1u), end = (int64_t)(uint32_t)(e - 1u);
    if (tid < 0 || tid >= P.n_targets || end <= beg) return sink.n;   // no reads (A3)
    const int64_t ra = P.tid_off[tid], rb = P.tid_off[tid + 1];
    const int32_t *pos = P.pos;
    const int32_t *emax = P.emax;
    int64_t hi = wave_partition_point(ra, rb, [&](int64_t r) { return (int64_t)pos[r] >= end; });
    int64_t lo = wave_partition_point(ra, hi, [&](int64_t r) { return (int64_t)emax[r] > beg; });
    const int ln = lane_id();
    for (int64_t base = lo; base < hi; base += WAVE) {
        int64_t r = base + ln;
        bool valid = r < hi;
        uint4 rc = valid ? P.rec[r] : make_uint4(0, 0, 0, 0);
        int32_t rp = valid ? pos[r] : 0;
        bool ov = valid && (int64_t)(int32_t)rc.x > beg;   // pos < end holds below hi (hts_itr_next)
        uint64_t m = ballot(ov);
        while (m) {
            int l = __builtin_ctzll(m);
            m &= m - 1;
            uint32_t rpos = rdlane((uint32_t)rp, l);
            uint32_t nc = rdlane(rc.y, l);
            uint64_t off = ((uint64_t)rdlane(rc.w, l) << 32) | rdlane(rc.z, l);
            walk_read<KIND, COUNT>(P.cigar, off, nc & 0x3fffffffu, rpos, nc >> 30, s, e, sink, st);
        }
    }
    return sink.n;
}

// Bitonic sort of buf[0..N) (N power of two, padded with INT32_MAX) by one wave.
__device__ void wave_bitonic_sort(int32_t *buf, int N) {
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
            __syncthreads();
        }
    }
}

__device__ __forceinline__ int32_t ref_abs(int32_t a) { return a < 0 ? -a : a; }   // refinement.h:41

// First index in [l, h) of sorted buf with buf[idx] > key  (per-lane binary search)
__device__ __forceinline__ int32_t first_greater(const int32_t *buf, int32_t l, int32_t h, int64_t key) {
    while (l < h) {
        int32_t m = (l + h) >> 1;
        if ((int64_t)buf[m] > key) h = m; else l = m + 1;
    }
    return l;
}
// First index in [l, h) with buf[idx] >= key
__device__ __forceinline__ int32_t first_geq(const int32_t *buf, int32_t l, int32_t h, int64_t key) {
    while (l < h) {
        int32_t m = (l + h) >> 1;
        if ((int64_t)buf[m] >= key) h = m; else l = m + 1;
    }
    return l;
}

__device__ __forceinline__ int32_t mean_round(int64_t tot, int32_t cnt) {
    // (int)((uint64 total + count/2) / count), refinement.c:66
    uint64_t t = (uint64_t)tot + (uint64_t)(int64_t)(cnt / 2);
    return (int32_t)(uint32_t)(t / (uint64_t)(int64_t)cnt);
}

// consensus_pos (refinement.c:41-101) on sorted A[0..n) with prefix sums P[0..n].
__device__ int32_t vote(const int32_t *A, const int64_t *P, int32_t n, int32_t pos, const KParams &k) {
    const int ln = lane_id();
    const int32_t ci = k.ci, range = k.range;
    int32_t valL = -1, maxL = k.min_count - 1, distL = 0x7fffffff;
    int32_t valR = -1, maxR = k.min_count - 1, distR = 0x7fffffff;

    // lower_bound(A, n, pos+25): (#elements <= pos+25) - 1, clamped at 0  (refinement.c:3-10)
    int32_t u = 0;
    for (int32_t b = 0; b < n; b += WAVE) {
        int32_t i = b + ln;
        u += __popcll(ballot(i < n && A[i] <= pos + SV_MIN_LENGTH / 2));
    }
    int32_t p = u == 0 ? 0 : u - 1;

    // left pass: i = p, p-1, ... while |pos - A[i]| < range   (refinement.c:58-77)
    for (int32_t top = p; top >= 0; top -= WAVE) {
        int32_t i = top - ln;
        bool inr = i >= 0 && ref_abs(pos - A[i < 0 ? 0 : i]) < range;
        uint64_t stop = ballot(!inr);
        int lim = stop ? __builtin_ctzll(stop) : WAVE;   // lanes [0, lim) are in the pass
        int32_t cnt = 0, cand = 0;
        if (ln < lim) {
            int32_t a = A[i];
            int32_t kk = first_geq(A, 0, i, (int64_t)a - ci);   // contiguous j<i with a <= A[j]+ci
            cnt = i - kk + 1;
            cand = mean_round(P[i + 1] - P[kk], cnt);
        }
        for (int l = 0; l < lim; l++) {
            int32_t c = rdlane_i(cnt, l), v = rdlane_i(cand, l);
            if (c > maxL) {
                int32_t d = ref_abs(pos - v);
                if (d < ci) return v;                    // early return, refinement.c:69-70
                if (d < distL) { maxL = c; valL = v; distL = d; }
            }
        }
        if (stop) break;
    }

    // upper_bound(A, n, pos-25): 0 if A[0] < pos-25 else n-1   (refinement.c:12-19)
    int32_t q = (n > 0 && A[0] < pos - SV_MIN_LENGTH / 2) ? 0 : n - 1;
    for (int32_t bot = q; bot < n; bot += WAVE) {
        int32_t i = bot + ln;
        bool inr = i < n && ref_abs(pos - A[i < n ? i : 0]) < range;
        uint64_t stop = ballot(!inr);
        int lim = stop ? __builtin_ctzll(stop) : WAVE;
        int32_t cnt = 0, cand = 0;
        if (ln < lim) {
            int32_t a = A[i];
            int32_t m = first_greater(A, i + 1, n, (int64_t)a + ci);   // contiguous j>i with A[j] <= a+ci
            cnt = m - i;
            cand = mean_round(P[m] - P[i], cnt);
        }
        for (int l = 0; l < lim; l++) {
            int32_t c = rdlane_i(cnt, l), v = rdlane_i(cand, l);
            if (c > maxR) {
                int32_t d = ref_abs(pos - v);
                if (d < ci) return v;
                if (d < distR) { maxR = c; valR = v; distR = d; }
            }
        }
        if (stop) break;
    }
    return distL < distR ? valL : valR;   // refinement.c:100
}

// Sort + prefix sums + vote over buf[0..n) with scratch for P (n+1 int64).
__device__ int32_t sort_and_vote(int32_t *buf, int64_t *P, int32_t n, int32_t pos, const KParams &k) {
    const int ln = lane_id();
    int N = 1;
    while (N < n) N <<= 1;
    for (int i = n + ln; i < N; i += WAVE) buf[i] = INT32_MAX;
    __syncthreads();
    wave_bitonic_sort(buf, N);
    int64_t carry = 0;
    if (ln == 0) P[0] = 0;
    for (int32_t b = 0; b < n; b += WAVE) {
        int32_t i = b + ln;
        int64_t x = i < n ? (int64_t)buf[i] : 0;
        int64_t s = carry + wave_scan_add64(x);
        if (i < n) P[i + 1] = s;
        carry = (int64_t)rdlane64((uint64_t)s, WAVE - 1);
    }
    __syncthreads();
    return vote(buf, P, n, pos, k);
}

template <int KIND, bool COUNT>
__device__ int32_t refine_window(const KArgs &a, int32_t *lds_c, int64_t *lds_p, int chrom, uint32_t s,
                                 uint32_t e, uint32_t imprecise, unsigned long long *wk) {
    WinStats<COUNT> st;
    Sink sink{lds_c, CAP, 0};
    int32_t n = gather_window<KIND, COUNT>(a.pile, chrom - 1, s, e, sink, st);
    if (COUNT && lane_id() == 0) {
        wk[0] += 1; wk[1] += st.reads; wk[2] += st.ops; wk[3] += (unsigned long long)n;
    }
    if (n < a.prm.min_count) return -1;                    // refinement.c:43-45
    if (n <= CAP) {
        __syncthreads();
        return sort_and_vote(lds_c, lds_p, n, (int32_t)imprecise, a.prm);
    }
    // spill: take a slab for N ints + (n+1) int64 from the device pool and re-gather
    if (COUNT && lane_id() == 0) wk[4] += 1;
    int N = 1;
    while (N < n) N <<= 1;
    unsigned long long words = (unsigned long long)N + 2ull * (unsigned long long)(n + 2);
    unsigned long long base = 0;
    if (lane_id() == 0) base = atomicAdd(a.pool_head, words);
    base = rdlane64(base, 0);
    if (base + words > a.pool_words) {
        if (lane_id() == 0) atomicOr(a.status, 1);
        return -1;
    }
    int32_t *g = a.pool + base;
    int64_t *gp = (int64_t *)(a.pool + ((base + (unsigned long long)N + 1ull) & ~1ull));
    WinStats<COUNT> st2;
    Sink s2{g, N, 0};
    gather_window<KIND, COUNT>(a.pile, chrom - 1, s, e, s2, st2);
    __syncthreads();
    return sort_and_vote(g, gp, n, (int32_t)imprecise, a.prm);
}

template <bool COUNT>
__global__ __launch_bounds__(64) void refine_kernel(KArgs a) {
    __shared__ int32_t lds_c[CAP];
    __shared__ int64_t lds_p[CAP + 1];
    const uint32_t li = blockIdx.x;
    if (li >= a.n) return;
    const svt_locus L = a.loci[li];
    const int32_t type = uniform_i(L.type), chrom = uniform_i(L.chrom);
    const uint32_t pos = (uint32_t)uniform_i((int32_t)L.pos), end = (uint32_t)uniform_i((int32_t)L.end);
    unsigned long long wk[5] = {0, 0, 0, 0, 0};
    uint32_t r0 = SVT_NA, r1 = SVT_NA;
    const KParams &k = a.prm;
    if (type == T_INS) {                                   // audit.c:176-187
        uint32_t s = pos - (uint32_t)k.median, e = pos + (uint32_t)k.median;
        r0 = (uint32_t)refine_window<K_INS, COUNT>(a, lds_c, lds_p, chrom, s, e, pos, wk);
    } else if (type == T_DEL) {                            // audit.c:188-220
        uint32_t bs = pos - (uint32_t)k.wider, be = pos + (uint32_t)k.narrow;
        uint32_t es = end - (uint32_t)k.narrow, ee = end + (uint32_t)k.narrow;
        r0 = (uint32_t)refine_window<K_START, COUNT>(a, lds_c, lds_p, chrom, bs, be, pos, wk);
        __syncthreads();
        r1 = (uint32_t)refine_window<K_END, COUNT>(a, lds_c, lds_p, chrom, es, ee, end, wk);
    }
    // INV: refine_point collects only when sv_type == SV_INS (refinement.c:250), so both
    // windows vote on 0 candidates -> -1 for every min_count >= 1 (validated): NA, NA.
    if (lane_id() == 0) {
        a.out[li] = svt_result{r0, r1};
        if (COUNT) {
            for (int i = 0; i < 5; i++)
                if (wk[i]) atomicAdd(a.work + i, wk[i]);
        }
    }
}

}  // namespace

// ====================================================================== C ABI
struct svt_ctx {
    svt_params prm{};
    int device = 0;
    char err[512] = {0};
    // pileup
    int32_t n_targets = 0;
    int64_t n_reads = 0;
    uint64_t n_ops = 0;
    int32_t *d_pos = nullptr, *d_emax = nullptr;
    uint4 *d_rec = nullptr;
    int64_t *d_tid_off = nullptr;
    uint32_t *d_cigar = nullptr;
    uint64_t dev_bytes = 0;
    bool loaded = false;
    // batch scratch
    svt_locus *d_loci = nullptr;
    svt_result *d_out = nullptr;
    size_t batch_cap = 0;
    // spill pool + status + work counters (one allocation, memset per call)
    int32_t *d_pool = nullptr;
    unsigned long long pool_words = 0;
    unsigned char *d_ctl = nullptr;   // [0,8) pool head, [8,12) status, [16,56) work
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

void free_pileup(svt_ctx *c) {
    (void)hipFree(c->d_pos); (void)hipFree(c->d_emax); (void)hipFree(c->d_rec); (void)hipFree(c->d_tid_off); (void)hipFree(c->d_cigar);
    c->d_pos = c->d_emax = nullptr; c->d_rec = nullptr; c->d_tid_off = nullptr; c->d_cigar = nullptr;
    c->loaded = false; c->dev_bytes = 0; c->n_reads = 0; c->n_ops = 0; c->n_targets = 0;
}

KArgs make_args(svt_ctx *c, const svt_locus *d_loci, svt_result *d_out, uint32_t n, bool count) {
    KArgs a;
    a.pile = DevPileup{c->d_pos, c->d_emax, c->d_rec, c->d_tid_off, c->d_cigar, c->n_targets};
    a.prm = KParams{c->prm.wider_interval, c->prm.median_interval, c->prm.narrow_interval,
                    c->prm.consensus_interval_range, c->prm.consensus_interval, c->prm.consensus_min_count};
    a.loci = d_loci;
    a.out = d_out;
    a.n = n;
    a.pool = c->d_pool;
    a.pool_head = (unsigned long long *)c->d_ctl;
    a.pool_words = c->pool_words;
    a.status = (int32_t *)(c->d_ctl + 8);
    a.work = count ? (unsigned long long *)(c->d_ctl + 16) : nullptr;
    return a;
}

svt_status launch(svt_ctx *c, const svt_locus *d_loci, svt_result *d_out, size_t n, hipStream_t st, bool count) {
    if (n == 0) return SVT_OK;
    if (n > 0x7fffffffull) return fail(c, SVT_EINVAL, "batch too large (%s)", "n > 2^31-1");
    HIP_TRY(c, hipMemsetAsync(c->d_ctl, 0, 64, st));
    KArgs a = make_args(c, d_loci, d_out, (uint32_t)n, count);
    if (count) hipLaunchKernelGGL(refine_kernel<true>, dim3((unsigned)n), dim3(64), 0, st, a);
    else hipLaunchKernelGGL(refine_kernel<false>, dim3((unsigned)n), dim3(64), 0, st, a);
    HIP_TRY(c, hipGetLastError());
    return SVT_OK;
}

svt_status ensure_batch(svt_ctx *c, size_t n) {
    if (n <= c->batch_cap) return SVT_OK;
    (void)hipFree(c->d_loci); (void)hipFree(c->d_out);
    c->d_loci = nullptr; c->d_out = nullptr; c->batch_cap = 0;
    HIP_TRY(c, hipMalloc(&c->d_loci, n * sizeof(svt_locus)));
    HIP_TRY(c, hipMalloc(&c->d_out, n * sizeof(svt_result)));
    c->batch_cap = n;
    return SVT_OK;
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
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) {
        delete c;
        return SVT_EDEVICE;
    }
    if (device >= 0) {
        if (device >= ndev || hipSetDevice(device) != hipSuccess) { delete c; return SVT_EDEVICE; }
        c->device = device;
    } else {
        (void)hipGetDevice(&c->device);
    }
    uint64_t pool_bytes = params->spill_bytes ? params->spill_bytes : (64ull << 20);
    c->pool_words = pool_bytes / 4;
    if (hipMalloc(&c->d_pool, c->pool_words * 4) != hipSuccess || hipMalloc(&c->d_ctl, 64) != hipSuccess) {
        (void)hipFree(c->d_pool);
        delete c;
        return SVT_ENOMEM;
    }
    (void)hipMemset(c->d_ctl, 0, 64);
    *out = c;
    return SVT_OK;
}

svt_status svt_load_pileup(svt_ctx *c, const svt_pileup_view *p) {
    if (!c || !p) return SVT_EINVAL;
    if (p->n_targets < 0 || (p->n_targets > 0 && !p->tid_off))
        return fail(c, SVT_EINVAL, "pileup: %s", "bad n_targets / tid_off");
    HIP_TRY(c, hipSetDevice(c->device));
    free_pileup(c);
    const int32_t nt = p->n_targets;
    const int64_t nr = nt ? p->tid_off[nt] : 0;
    if (nt && p->tid_off[0] != 0) return fail(c, SVT_EINVAL, "pileup: %s", "tid_off[0] != 0");
    for (int32_t t = 0; t < nt; t++)
        if (p->tid_off[t + 1] < p->tid_off[t]) return fail(c, SVT_EINVAL, "pileup: %s", "tid_off not monotone");
    if (nr > 0 && (!p->pos || !p->endpos || !p->cig_off || (!p->cigar && p->cig_off[nr] > 0)))
        return fail(c, SVT_EINVAL, "pileup: %s", "missing arrays");
    const uint64_t nops = nr > 0 ? p->cig_off[nr] : 0;
    if (nr > 0 && p->cig_off[0] != 0) return fail(c, SVT_EINVAL, "pileup: %s", "cig_off[0] != 0");

    std::vector<int32_t> emax((size_t)nr);
    std::vector<uint4> rec((size_t)nr);
    for (int32_t t = 0; t < nt; t++) {
        int32_t m = INT32_MIN;
        for (int64_t r = p->tid_off[t]; r < p->tid_off[t + 1]; r++) {
            if (r > p->tid_off[t] && p->pos[r] < p->pos[r - 1])
                return fail(c, SVT_EINVAL, "pileup: %s", "reads not sorted by pos within a contig");
            if (p->pos[r] < 0 || p->endpos[r] <= p->pos[r])
                return fail(c, SVT_EINVAL, "pileup: %s", "pos < 0 or endpos <= pos");
            uint64_t o0 = p->cig_off[r], o1 = p->cig_off[r + 1];
            if (o1 < o0 || o1 > nops || o1 - o0 >= (1ull << 30))
                return fail(c, SVT_EINVAL, "pileup: %s", "bad cig_off");
            uint32_t ncig = (uint32_t)(o1 - o0);
            uint32_t clip;
            if (p->clip) clip = p->clip[r] & 3u;
            else clip = ncig ? (((p->cigar[o1 - 1] & 0xfu) == OP_SOFT ? 1u : 0u) |
                                ((p->cigar[o0] & 0xfu) == OP_SOFT ? 2u : 0u)) : 0u;
            if (p->endpos[r] > m) m = p->endpos[r];
            emax[(size_t)r] = m;
            rec[(size_t)r] = make_uint4((uint32_t)p->endpos[r], ncig | (clip << 30), (uint32_t)o0,
                                        (uint32_t)(o0 >> 32));
        }
    }
    size_t nrs = (size_t)(nr > 0 ? nr : 1);
    HIP_TRY(c, hipMalloc(&c->d_pos, nrs * 4));
    HIP_TRY(c, hipMalloc(&c->d_emax, nrs * 4));
    HIP_TRY(c, hipMalloc(&c->d_rec, nrs * 16));
    HIP_TRY(c, hipMalloc(&c->d_tid_off, (size_t)(nt + 1) * 8));
    HIP_TRY(c, hipMalloc(&c->d_cigar, (size_t)(nops > 0 ? nops : 1) * 4));
    if (nr > 0) {
        HIP_TRY(c, hipMemcpy(c->d_pos, p->pos, (size_t)nr * 4, hipMemcpyHostToDevice));
        HIP_TRY(c, hipMemcpy(c->d_emax, emax.data(), (size_t)nr * 4, hipMemcpyHostToDevice));
        HIP_TRY(c, hipMemcpy(c->d_rec, rec.data(), (size_t)nr * 16, hipMemcpyHostToDevice));
    }
    if (nt > 0) HIP_TRY(c, hipMemcpy(c->d_tid_off, p->tid_off, (size_t)(nt + 1) * 8, hipMemcpyHostToDevice));
    else HIP_TRY(c, hipMemset(c->d_tid_off, 0, 8));
    if (nops > 0) HIP_TRY(c, hipMemcpy(c->d_cigar, p->cigar, nops * 4, hipMemcpyHostToDevice));
    c->n_targets = nt;
    c->n_reads = nr;
    c->n_ops = nops;
    c->dev_bytes = (uint64_t)nr * 24 + (uint64_t)(nt + 1) * 8 + nops * 4;
    c->loaded = true;
    return SVT_OK;
}

svt_status svt_refine_device(svt_ctx *c, const svt_locus *d_loci, size_t n, svt_result *d_out, void *stream) {
    if (!c) return SVT_EINVAL;
    if (!c->loaded) return fail(c, SVT_ESTATE, "%s", "svt_load_pileup not called");
    if (n && (!d_loci || !d_out)) return fail(c, SVT_EINVAL, "%s", "null loci/out");
    return launch(c, d_loci, d_out, n, (hipStream_t)stream, false);
}

svt_status svt_sync(svt_ctx *c, void *stream) {
    if (!c) return SVT_EINVAL;
    HIP_TRY(c, hipStreamSynchronize((hipStream_t)stream));
    int32_t status = 0;
    HIP_TRY(c, hipMemcpy(&status, c->d_ctl + 8, 4, hipMemcpyDeviceToHost));
    if (status & 1) return fail(c, SVT_EOVERFLOW, "%s", "candidate spill pool exhausted (raise spill_bytes)");
    return SVT_OK;
}

svt_status svt_refine_batch(svt_ctx *c, const svt_locus *loci, size_t n, svt_result *out) {
    if (!c) return SVT_EINVAL;
    if (!c->loaded) return fail(c, SVT_ESTATE, "%s", "svt_load_pileup not called");
    if (n == 0) return SVT_OK;
    if (!loci || !out) return fail(c, SVT_EINVAL, "%s", "null loci/out");
    HIP_TRY(c, hipSetDevice(c->device));
    svt_status s = ensure_batch(c, n);
    if (s) return s;
    HIP_TRY(c, hipMemcpy(c->d_loci, loci, n * sizeof(svt_locus), hipMemcpyHostToDevice));
    s = launch(c, c->d_loci, c->d_out, n, nullptr, false);
    if (s) return s;
    s = svt_sync(c, nullptr);
    if (s) return s;
    HIP_TRY(c, hipMemcpy(out, c->d_out, n * sizeof(svt_result), hipMemcpyDeviceToHost));
    return SVT_OK;
}

svt_status svt_count_work(svt_ctx *c, const svt_locus *loci, size_t n, svt_work *out) {
    if (!c || !out) return SVT_EINVAL;
    if (!c->loaded) return fail(c, SVT_ESTATE, "%s", "svt_load_pileup not called");
    memset(out, 0, sizeof(*out));
    if (n == 0) return SVT_OK;
    HIP_TRY(c, hipSetDevice(c->device));
    svt_status s = ensure_batch(c, n);
    if (s) return s;
    HIP_TRY(c, hipMemcpy(c->d_loci, loci, n * sizeof(svt_locus), hipMemcpyHostToDevice));
    s = launch(c, c->d_loci, c->d_out, n, nullptr, true);
    if (s) return s;
    s = svt_sync(c, nullptr);
    if (s) return s;
    unsigned long long w[5];
    HIP_TRY(c, hipMemcpy(w, c->d_ctl + 16, sizeof w, hipMemcpyDeviceToHost));
    out->windows = w[0]; out->reads = w[1]; out->ops_walked = w[2]; out->candidates = w[3];
    out->spilled_windows = w[4];
    return SVT_OK;
}

uint64_t svt_pileup_device_bytes(const svt_ctx *c) { return c ? c->dev_bytes : 0; }

void svt_close(svt_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    free_pileup(c);
    (void)hipFree(c->d_loci); (void)hipFree(c->d_out); (void)hipFree(c->d_pool); (void)hipFree(c->d_ctl);
    delete c;
}

}  // extern "C"
