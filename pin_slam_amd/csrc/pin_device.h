// pin_device.h -- device-side building blocks shared by the gfx950 kernels.
//
// Numerics: the library is compiled with -ffp-contract=off so that every
// elementwise expression rounds like the reference's unfused ATen ops
// (voxel floor, squared distance, IDW weights).  FMAs are written explicitly
// (fmaf) only inside the MLP dot products, whose order the reference leaves to BLAS.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pin_slam_amd.h"

// Tuning switches (compile-time; tools/variants.py sweeps them)
#ifndef PIN_MLP_UNROLL
#define PIN_MLP_UNROLL 2     // hidden-unit pairs per decoder-loop iteration
#endif
#ifndef PIN_NB_GROUP
#define PIN_NB_GROUP 4       // neighbours gathered per streaming group
#endif
#ifndef PIN_GRID_CHUNK
#define PIN_GRID_CHUNK 8     // candidate records fetched per round trip (grid source; 8 measured best, see DESIGN)
#endif

namespace pin {

constexpr int kF = PIN_FEATURE_DIM;      // feature_dim
constexpr int kD = kF + 3;               // decoder input: feature + neighbour vector
constexpr int kH = PIN_HIDDEN_DIM;       // geo_mlp_hidden_dim
constexpr int kK = PIN_MAX_NN_K;         // top-k capacity
#ifndef PIN_BLOCK
#define PIN_BLOCK 256
#endif
constexpr int kBlock = PIN_BLOCK;   // threads per block of the per-row kernels
constexpr int kIdMask = PIN_RECORD_UNFAITHFUL - 1;
constexpr int64_t kP0 = 73856093LL, kP1 = 19349669LL, kP2 = 83492791LL;  // neural_points.py:69
constexpr float kInvalidDist2 = 9e3f;    // neural_points.py:561
constexpr float kIdwEps = 1e-15f;        // neural_points.py:618

// XCD-aware block order: the hardware places block b on XCD (b mod 8); this bijection hands
// each XCD one contiguous eighth of the logical blocks, so spatially ordered inputs keep their
// neighbourhoods within one XCD's L2.
__device__ __forceinline__ int64_t xcd_block() {
    const int64_t nb = gridDim.x, b = blockIdx.x;
    const int64_t q = nb >> 3, r = nb & 7, x = b & 7;
    return x * q + (x < r ? x : r) + (b >> 3);
}

// floor_mod(floor(q/res) . primes, B): the reference's fmod + negative-index wrap
// (neural_points.py:465-476).  Division is IEEE f32 (no reciprocal), as on the CPU path.
__device__ __forceinline__ uint32_t base_slot(float qx, float qy, float qz, float res, int64_t B) {
    const int64_t gx = (int64_t)floorf(qx / res);
    const int64_t gy = (int64_t)floorf(qy / res);
    const int64_t gz = (int64_t)floorf(qz / res);
    const int64_t h = gx * kP0 + gy * kP1 + gz * kP2;
    int64_t r = h % B;
    if (r < 0) r += B;
    return (uint32_t)r;
}

// squared distance, reference op order: ((dx*dx + dy*dy) + dz*dz) with d = p - q (:492-495)
__device__ __forceinline__ float dist2(float px, float py, float pz, float qx, float qy, float qz) {
    const float dx = px - qx, dy = py - qy, dz = pz - qz;
    return (dx * dx + dy * dy) + dz * dz;
}

#ifndef PIN_TOPK_MED3
#define PIN_TOPK_MED3 1   // 0: the two-select form of the distance update (experiment switch)
#endif

// Sorted (ascending) register list of the k nearest candidates.  Ties keep candidate
// order (cell order); a list with a tie is redone in the reference's order (resolve_ties).
struct TopK {
    float d[kK];
    int g[kK];
    float rej;   // the smallest distance that did not stay in the list (tie check, resolve_ties)
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int j = 0; j < kK; ++j) { d[j] = kInvalidDist2; g[j] = -1; }
        rej = INFINITY;
    }
    // Branch-free insertion (pure selects).  x = +inf is a no-op, so callers insert every
    // candidate unconditionally with rejected ones mapped to +inf.
    // The distances take one v_med3 each: with d ascending, the selected value
    // c[j] ? d[j] : (c[j-1] ? x : d[j-1]) is the median of (d[j-1], x, d[j]) (equal values are
    // interchangeable, so ties change nothing); the payloads keep the two selects.
    __device__ __forceinline__ void insert(float x, int gi) {
        // the smaller of rej and what leaves the list (x itself, or the entry x pushes out):
        // rej >= d[kK-1] always, so that is the median of (d[kK-1], x, rej) -- one v_med3
        rej = __builtin_amdgcn_fmed3f(d[kK - 1], x, rej);
        bool c[kK];
#pragma unroll
        for (int j = 0; j < kK; ++j) c[j] = d[j] <= x;
#pragma unroll
        for (int j = kK - 1; j > 0; --j) {
            const int gj = c[j - 1] ? gi : g[j - 1];
#if PIN_TOPK_MED3
            d[j] = __builtin_amdgcn_fmed3f(d[j - 1], x, d[j]);
#else
            d[j] = c[j] ? d[j] : (c[j - 1] ? x : d[j - 1]);
#endif
            g[j] = c[j] ? g[j] : gj;
        }
        d[0] = c[0] ? d[0] : x;
        g[0] = c[0] ? g[0] : gi;
    }
};

// Pair mode (two lanes per query, the even lane's candidates before the odd lane's in the
// reference order): both lanes end with the even lane's list and the odd lane's candidates
// inserted after it -- the sequential scan's result, ties included (insert keeps arrival order).
__device__ __forceinline__ void topk_pair_merge(TopK& tk, int ph) {
    float od[kK];
    int og[kK];
#pragma unroll
    for (int j = 0; j < kK; ++j) {
        od[j] = __shfl_xor(tk.d[j], 1);
        og[j] = __shfl_xor(tk.g[j], 1);
    }
    TopK base;
    float ad[kK];
    int ag[kK];
#pragma unroll
    for (int j = 0; j < kK; ++j) {
        base.d[j] = ph ? od[j] : tk.d[j];
        base.g[j] = ph ? og[j] : tk.g[j];
        ad[j] = ph ? tk.d[j] : od[j];
        ag[j] = ph ? tk.g[j] : og[j];
    }
    base.rej = fminf(tk.rej, __shfl_xor(tk.rej, 1));
#pragma unroll
    for (int j = 0; j < kK; ++j) base.insert(ad[j], ag[j]);
    tk = base;
}

// ---------------------------------------------------------------------------------------
// Equal distances.  The reference orders a query's Kc candidate distances with torch's CPU
// sort(stable=False) (model/neural_points.py:561-565), which is libstdc++'s std::sort over the
// row (aten SortingKernel), and keeps the first k.  Where two VALID candidates have exactly the
// same distance the order std::sort leaves them in is not cell order: it depends on the whole
// row (median-of-three pivots, partitions, the final insertion sort).  Lattice-quantised scans
// make exact ties frequent enough to matter: taking them in cell order (a stable sort) prefers
// the cells of lower offsets.  The streaming top-k above keeps cell order;
// a query whose kept list has a tie is redone in the reference's order by its WAVE
// (resolve_ties): the row of Kc (distance, payload) pairs, 9e3 for the invalid ones as in the
// reference, held two entries per lane in registers (no private memory, no LDS), sorted by a
// wave-parallel restatement of std::sort, and its first entries handed to the query's lane.
//
// Which ties: a tie at the k-th place (between the k-th kept candidate and the first one left
// out) changes the neighbour SET -- the hot kernels resolve those (kTieBoundary); ties inside the
// kept list only change the order of the neighbours, i.e. the summation order of the IDW sums,
// which matters where the order is an output (query_feature's per-neighbour layout, kTieAll).
constexpr int kRefSortMax = 128;   // rows up to this many cells (Kc <= 125 with num_nei_cells 2)
enum TieScope { kTieBoundary = 0, kTieAll = 1 };

#ifndef PIN_REF_TIES
#define PIN_REF_TIES 1   // 0: keep cell order for equal distances (experiment switch)
#endif

__device__ __forceinline__ bool topk_tied(const TopK& tk, int nn_k, int nn, TieScope scope) {
    bool t = false;
    if (scope == kTieAll) {
#pragma unroll
        for (int j = 0; j + 1 < kK; ++j)
            t = t || (j + 1 < nn_k && j + 1 < nn && tk.d[j] == tk.d[j + 1]);
    }
    // the k-th place: against the (k+1)-th candidate, kept in the list or (k == kK) the best
    // one pushed out of it
    if (nn_k < kK) {
#pragma unroll
        for (int j = 1; j < kK; ++j)
            t = t || (j == nn_k && nn > nn_k && tk.d[j - 1] == tk.d[j]);
    } else {
        t = t || (nn > kK && tk.rej == tk.d[kK - 1]);
    }
    return t;
}

// A row of up to 128 (key, payload) entries held by the wave: lane l has entry l in (ka, ga) and
// entry l + 64 in (kb, gb).  Entry reads and writes at a wave-uniform position use readlane /
// a lane select; permutations use ds_bpermute.  All 64 lanes must be active.
struct WaveRow {
    float ka, kb;
    int ga, gb;
};

__device__ __forceinline__ int wave_lane() { return threadIdx.x & 63; }
__device__ __forceinline__ float rdl_f(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float row_key(const WaveRow& r, int p) { return p < 64 ? rdl_f(r.ka, p) : rdl_f(r.kb, p - 64); }
__device__ __forceinline__ int row_pay(const WaveRow& r, int p) {
    return p < 64 ? __builtin_amdgcn_readlane(r.ga, p) : __builtin_amdgcn_readlane(r.gb, p - 64);
}
__device__ __forceinline__ void row_set(WaveRow& r, int p, float k, int g) {
    const int lane = wave_lane();
    const bool a = p < 64 && lane == p, b = p >= 64 && lane == p - 64;
    r.ka = a ? k : r.ka;
    r.ga = a ? g : r.ga;
    r.kb = b ? k : r.kb;
    r.gb = b ? g : r.gb;
}
__device__ __forceinline__ void row_swap(WaveRow& r, int p, int q) {
    const float kp = row_key(r, p), kq = row_key(r, q);
    const int gp = row_pay(r, p), gq = row_pay(r, q);
    row_set(r, p, kq, gq);
    row_set(r, q, kp, gp);
}
// new entry p = old entry src(p): sa for the lane's entry in .a, sb for its entry in .b
__device__ __forceinline__ void row_gather(WaveRow& r, int sa, int sb) {
    const float ka_a = __shfl(r.ka, sa & 63), kb_a = __shfl(r.kb, sa & 63);
    const int ga_a = __shfl(r.ga, sa & 63), gb_a = __shfl(r.gb, sa & 63);
    const float ka_b = __shfl(r.ka, sb & 63), kb_b = __shfl(r.kb, sb & 63);
    const int ga_b = __shfl(r.ga, sb & 63), gb_b = __shfl(r.gb, sb & 63);
    r.ka = sa < 64 ? ka_a : kb_a;
    r.ga = sa < 64 ? ga_a : gb_a;
    r.kb = sb < 64 ? ka_b : kb_b;
    r.gb = sb < 64 ? ga_b : gb_b;
}

// 128-bit position masks (lo: entries 0..63, hi: 64..127)
__device__ __forceinline__ uint64_t mask_upto(int b) {   // bits 0..b (b in [-1, 63])
    return b < 0 ? 0ull : (b >= 63 ? ~0ull : ((2ull << b) - 1ull));
}
__device__ __forceinline__ int count_upto(uint64_t lo, uint64_t hi, int p) {   // set bits at positions <= p
    return p < 64 ? __popcll(lo & mask_upto(p)) : __popcll(lo) + __popcll(hi & mask_upto(p - 64));
}
// position of the t-th set bit from the low end (t >= 1), 128 if there is none
__device__ __forceinline__ int select_low(uint64_t lo, uint64_t hi, int t) {
    uint64_t m = lo;
    int base = 0;
    const int cl = __popcll(lo);
    if (t > cl) {
        t -= cl;
        m = hi;
        base = 64;
        if (t > __popcll(hi)) return 128;
    }
    int pos = 0;   // invariant: fewer than t set bits below pos
#pragma unroll
    for (int s = 32; s > 0; s >>= 1)
        if (__popcll(m & mask_upto(pos + s - 1)) < t) pos += s;
    return base + pos;
}
// position of the u-th set bit from the high end (u >= 1), -1 if there is none
__device__ __forceinline__ int select_high(uint64_t lo, uint64_t hi, int u) {
    const int tot = __popcll(lo) + __popcll(hi);
    return u > tot ? -1 : select_low(lo, hi, tot - u + 1);
}

// libstdc++ __unguarded_partition(first + 1, last, first) on entries [f, l) with the pivot at f,
// all swaps at once: with L_t the t-th entry from the left that is not below the pivot and R_t
// the t-th from the right that is not above it (both in the row as it was), the sequential scans
// swap L_t with R_t for every t with L_t < R_t (s pairs: their positions never overlap, and each
// scan only crosses entries the earlier swaps left untouched) and return min(L_{s+1}, R_s)
// (L_1 when s = 0).  Returns the cut.
__device__ __forceinline__ int wave_partition(WaveRow& r, int f, int l) {
    const int pa = wave_lane(), pb = pa + 64;
    const float pv = row_key(r, f);
    const bool ina = pa > f && pa < l, inb = pb > f && pb < l;
    const bool gea = ina && !(r.ka < pv), geb = inb && !(r.kb < pv);
    const bool lea = (ina || pa == f) && !(pv < r.ka), leb = (inb || pb == f) && !(pv < r.kb);
    const uint64_t geLo = __ballot(gea), geHi = __ballot(geb);
    const uint64_t leLo = __ballot(lea), leHi = __ballot(leb);
    const int leTot = __popcll(leLo) + __popcll(leHi);
    // left rank of a left stop, its partner R_t; swaps happen for L_t < R_t
    const int ta = count_upto(geLo, geHi, pa), tb = count_upto(geLo, geHi, pb);
    const int rta = gea ? select_high(leLo, leHi, ta) : -1, rtb = geb ? select_high(leLo, leHi, tb) : -1;
    const bool swa = gea && pa < rta, swb = geb && pb < rtb;
    const int s = __popcll(__ballot(swa)) + __popcll(__ballot(swb));
    // right rank of a right stop (entries at or above it), its partner L_u
    const int ua = leTot - count_upto(leLo, leHi, pa - 1), ub = leTot - count_upto(leLo, leHi, pb - 1);
    const bool rsa = !swa && lea && ua <= s, rsb = !swb && leb && ub <= s;
    const int sa = swa ? rta : (rsa ? select_low(geLo, geHi, ua) : pa);
    const int sb = swb ? rtb : (rsb ? select_low(geLo, geHi, ub) : pb);
    row_gather(r, sa, sb);
    int cut = select_low(geLo, geHi, s + 1);
    if (s > 0) {
        const int rs = select_high(leLo, leHi, s);
        cut = cut < rs ? cut : rs;
    }
    if (cut > l) cut = l;   // unreachable: the median of three guarantees a left stop
    return __builtin_amdgcn_readfirstlane(cut);
}

// libstdc++ __adjust_heap + __push_heap / __make_heap + __sort_heap on [f, l): the depth-limit
// fallback, run entry by entry at wave-uniform positions (rare: needs a badly split row)
__device__ void wave_adjust_heap(WaveRow& r, int f, int h, int len, float vk, int vg) {
    const int top = h;
    int c = h;
    while (c < (len - 1) / 2) {
        c = 2 * (c + 1);
        if (row_key(r, f + c) < row_key(r, f + c - 1)) --c;
        row_set(r, f + h, row_key(r, f + c), row_pay(r, f + c));
        h = c;
    }
    if ((len & 1) == 0 && c == (len - 2) / 2) {
        c = 2 * (c + 1);
        row_set(r, f + h, row_key(r, f + c - 1), row_pay(r, f + c - 1));
        h = c - 1;
    }
    int parent = (h - 1) / 2;
    while (h > top && row_key(r, f + parent) < vk) {
        row_set(r, f + h, row_key(r, f + parent), row_pay(r, f + parent));
        h = parent;
        parent = (h - 1) / 2;
    }
    row_set(r, f + h, vk, vg);
}
__device__ void wave_heap_sort(WaveRow& r, int f, int l) {
    const int len = l - f;
    if (len >= 2) {
        for (int parent = (len - 2) / 2;; --parent) {
            wave_adjust_heap(r, f, parent, len, row_key(r, f + parent), row_pay(r, f + parent));
            if (parent == 0) break;
        }
    }
    while (l - f > 1) {
        --l;
        const float vk = row_key(r, l);
        const int vg = row_pay(r, l);
        row_set(r, l, row_key(r, f), row_pay(r, f));
        wave_adjust_heap(r, f, 0, l - f, vk, vg);
    }
}

// std::sort(row, row + n) (libstdc++: __introsort_loop with depth 2 floor(log2 n) and runs of 16,
// then __final_insertion_sort), then the first kK entries.  The loop's recursion on the right
// part is a stack of disjoint segments held one per lane (the order segments are finished in does
// not change the result).  The final insertion sort moves an entry left past strictly greater
// keys only, so it is the stable sort of the row the loop leaves: entry p lands at
// #(keys < k_p) + #(equal keys before p).  out_d / out_g: the k first keys / payloads, uniform.
__device__ void wave_introsort_loop(WaveRow& r, int n) {
    const int lane = wave_lane();
    int sF = 0, sL = 0, sD = 0;   // segment stack, entry e in lane e
    int top = 0;
    if (n > 16) {
        sF = lane == 0 ? 0 : sF;
        sL = lane == 0 ? n : sL;
        sD = lane == 0 ? 2 * (31 - __clz(n)) : sD;
        top = 1;
    }
    while (top > 0) {
        --top;
        int f = __builtin_amdgcn_readlane(sF, top), l = __builtin_amdgcn_readlane(sL, top);
        int depth = __builtin_amdgcn_readlane(sD, top);
        while (l - f > 16) {
            if (depth == 0) {
                wave_heap_sort(r, f, l);
                break;
            }
            --depth;
            // __move_median_to_first(f, f + 1, mid, l - 1)
            const int a = f + 1, b = f + (l - f) / 2, c = l - 1;
            const float ka = row_key(r, a), kb = row_key(r, b), kc = row_key(r, c);
            const int m = ka < kb ? (kb < kc ? b : (ka < kc ? c : a)) : (ka < kc ? a : (kb < kc ? c : b));
            row_swap(r, f, m);
            const int cut = wave_partition(r, f, l);
            sF = lane == top ? cut : sF;   // __introsort_loop(cut, last, depth)
            sL = lane == top ? l : sL;
            sD = lane == top ? depth : sD;
            ++top;
            l = cut;
        }
    }
}

// where the final insertion sort puts the lane's two entries (ra for entry lane, rb for lane + 64)
__device__ __forceinline__ void wave_final_rank(const WaveRow& r, int n, int& ra, int& rb) {
    const int pa = wave_lane(), pb = pa + 64;
    ra = 0;
    rb = 0;
    for (int q = 0; q < n; ++q) {
        const float kq = row_key(r, q);
        ra += (kq < r.ka || (kq == r.ka && q < pa)) ? 1 : 0;
        rb += (kq < r.kb || (kq == r.kb && q < pb)) ? 1 : 0;
    }
}

__device__ void wave_ref_sort(WaveRow& r, int n, float (&out_d)[kK], int (&out_g)[kK]) {
    wave_introsort_loop(r, n);
    const int pa = wave_lane(), pb = pa + 64;
    int ra, rb;
    wave_final_rank(r, n, ra, rb);
#pragma unroll
    for (int j = 0; j < kK; ++j) {
        const uint64_t ma = __ballot(pa < n && ra == j), mb = __ballot(pb < n && rb == j);
        const bool hasA = ma != 0ull, hasB = mb != 0ull;
        const int src = hasA ? (int)__builtin_ctzll(ma) : (hasB ? (int)__builtin_ctzll(mb) + 64 : -1);
        const float d = src >= 0 ? row_key(r, src) : kInvalidDist2;
        const int g = src >= 0 ? row_pay(r, src) : -1;
        const bool in = d < kInvalidDist2;
        out_d[j] = in ? d : kInvalidDist2;
        out_g[j] = in ? g : -1;
    }
}

// The reference's k first entries for every lane of the wave whose list has a tie in `scope`;
// src.ref_cell(q, c, key, payload) gives cell c's candidate (9e3 / -1 where the reference has
// idx -1).  Called by ALL lanes of the wave at the same point (the kernels run whole waves;
// a wave with inactive lanes keeps cell order, which only the last partial wave of a launch can
// be, and only when a rank's batch is not a multiple of 64).
template <class Src>
__device__ __forceinline__ void resolve_ties(const Src& src, float qx, float qy, float qz, int nn_k, int nn,
                                             TopK& tk, TieScope scope = kTieBoundary) {
    if (!PIN_REF_TIES) return;
    uint64_t m = __ballot(topk_tied(tk, nn_k, nn, scope));
    if (m == 0ull) return;
    if (__ballot(true) != ~0ull) return;
    const int n = src.num_cells();
    if (n > kRefSortMax) return;   // larger neighbourhoods keep cell order
    const int lane = wave_lane();
    while (m) {
        const int L = (int)__builtin_ctzll(m);
        m &= m - 1ull;
        const float x = rdl_f(qx, L), y = rdl_f(qy, L), z = rdl_f(qz, L);
        WaveRow r;
        src.ref_cell(x, y, z, lane, n, r.ka, r.ga);
        src.ref_cell(x, y, z, lane + 64, n, r.kb, r.gb);
        float d[kK];
        int g[kK];
        wave_ref_sort(r, n, d, g);
        if (lane == L) {
#pragma unroll
            for (int j = 0; j < kK; ++j) {
                tk.d[j] = d[j];
                tk.g[j] = g[j];
            }
        }
    }
}

// ---------------------------------------------------------------------------------------
// Candidate sources.  Both enumerate the neighbour cells of q in the reference's cell order
// (model/neural_points.py:430-439), reject empty / filtered / too-far candidates, keep the
// k nearest in a TopK whose payload is source specific, and return nn_count (valid
// candidates before truncation, :557).  Latency structure per chunk of CH cells: the CH
// cell lookups are issued back to back, then the CH record gathers are issued back to back
// with clamped (never branched) addresses -- an empty cell reads entry 0, a hot line -- so
// each chunk costs two memory round trips, not 2*CH.

// The reference structure: hash every neighbour cell into the slot table (:465-476).
// Payload = global point index; records indexed by it.
struct HashSource {
    static constexpr int kChunk = 12;
    static constexpr bool kIdPayload = false;
    const PinHash& h;
    const PinPoints& p;
    __device__ HashSource(const PinHash& h_, const PinPoints& p_) : h(h_), p(p_) {}

    template <int CH>
    __device__ __forceinline__ int scan(float qx, float qy, float qz, TopK& tk) const {
        const float4* __restrict__ rec = (const float4*)p.records;
        const uint32_t B = (uint32_t)h.buffer_size;
        const uint32_t base = base_slot(qx, qy, qz, h.resolution, h.buffer_size);
        const float maxd2 = h.max_valid_dist2;
        const int Kc = h.num_cells;
        const int32_t* __restrict__ delta = h.cells;  // padded to a multiple of 16 entries
        const int32_t* __restrict__ table = h.table;
        int nn = 0;
        for (int c0 = 0; c0 < Kc; c0 += CH) {
            int dl[CH];
#pragma unroll
            for (int t = 0; t < CH; ++t) dl[t] = delta[c0 + t];
            int gi[CH];
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                uint32_t s = base + (uint32_t)dl[t];
                s = s >= B ? s - B : s;
                gi[t] = (c0 + t < Kc) ? table[s] : -1;
            }
            float4 r[CH];
#pragma unroll
            for (int t = 0; t < CH; ++t) r[t] = rec[gi[t] > 0 ? gi[t] : 0];
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const int id = __float_as_int(r[t].w);
                const float d2 = dist2(r[t].x, r[t].y, r[t].z, qx, qy, qz);
                const bool ok = gi[t] >= 0 && id != -1 && d2 <= maxd2;
                nn += ok ? 1 : 0;
                tk.insert(ok ? d2 : INFINITY, gi[t]);
            }
        }
        return nn;
    }
    // one cell of the reference's sort row (resolve_ties): cell c's candidate distance and
    // payload, 9e3 / -1 where the reference has idx -1 (c >= n: an unused entry)
    __device__ __forceinline__ int num_cells() const { return h.num_cells; }
    __device__ __forceinline__ void ref_cell(float qx, float qy, float qz, int c, int n, float& k, int& g) const {
        const float4* __restrict__ rec = (const float4*)p.records;
        const uint32_t B = (uint32_t)h.buffer_size;
        const uint32_t base = base_slot(qx, qy, qz, h.resolution, h.buffer_size);
        uint32_t s = base + (uint32_t)h.cells[c < n ? c : 0];
        s = s >= B ? s - B : s;
        const int gi = c < n ? h.table[s] : -1;
        const float4 v = rec[gi > 0 ? gi : 0];
        const float d2 = dist2(v.x, v.y, v.z, qx, qy, qz);
        const bool ok = gi >= 0 && __float_as_int(v.w) != -1 && d2 <= h.max_valid_dist2;
        k = ok ? d2 : kInvalidDist2;
        g = ok ? gi : -1;
    }
    __device__ __forceinline__ float4 record(int pay) const { return ((const float4*)p.records)[pay > 0 ? pay : 0]; }
    __device__ __forceinline__ void features(int pay, int64_t id, float4& f0, float4& f1) const {
        const float4* __restrict__ feat = (const float4*)p.features;
        f0 = feat[2 * id];
        f1 = feat[2 * id + 1];
    }
    __device__ __forceinline__ float certainty(int pay, int64_t id) const { return p.certainties[id]; }
    __device__ __forceinline__ int gid(int pay) const { return pay; }
};

// The occupancy grid (pin_grid.hip): cell -> brick bit -> rank -> 64-byte compact record.
// Payload = compact record index.  FAT: features / certainty come from the compact record
// (one line per candidate); otherwise from the live PinPoints arrays.
// one of 8 registers by a per-lane 3-bit index, as a select tree (no scratch)
__device__ __forceinline__ uint32_t sel4v(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, int k);
__device__ __forceinline__ uint32_t sel8(const uint32_t (&w)[8], int k) {
    const uint32_t lo = sel4v(w[0], w[1], w[2], w[3], k), hi = sel4v(w[4], w[5], w[6], w[7], k);
    return (k & 4) ? hi : lo;
}

// one of 4 registers by a per-lane 2-bit index
__device__ __forceinline__ uint32_t sel4(const uint32_t* w, int k) {
    const uint32_t a0 = (k & 1) ? w[1] : w[0], a1 = (k & 1) ? w[3] : w[2];
    return (k & 2) ? a1 : a0;
}

// The same on four values.  Callers that pick between two register quads must select the
// VALUES (sel4v of each quad, then a select): a pointer select (w vs w + 4) makes the compiler
// spill the array to scratch and index it there -- a vector-memory round trip per lookup.
__device__ __forceinline__ uint32_t sel4v(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, int k) {
    const uint32_t a0 = (k & 1) ? w1 : w0, a1 = (k & 1) ? w3 : w2;
    return (k & 2) ? a1 : a0;
}

// Per-wave LDS list of the grid scan, [slot][lane] (one column per lane: conflict-free, no
// barrier).  The matrix-core decoder takes the wave's slice as its scratch once the wave's scan
// is over (mlp_sdf_mfma16), so the two share 32 KB per block.
#ifndef PIN_LIST_SEG
#define PIN_LIST_SEG 32
#endif
constexpr int kListSeg = PIN_LIST_SEG;   // offsets per list segment
// the block's lists, contiguous: after a block barrier a kernel may reuse all of it (block_list)
__device__ __forceinline__ int* block_list() {
    __shared__ int s_list[kBlock / 64][kListSeg * 64];
    return &s_list[0][0];
}
__device__ __forceinline__ int* wave_list() { return block_list() + (threadIdx.x >> 6) * (kListSeg * 64); }

// IDP: the top-k payload is the record's feature-row id (flags stripped) instead of its
// compact index -- for the training forward, which reads features and positions by id and never
// needs the record again (one dependent round trip fewer per neighbour group).
template <bool FAT, bool IDP = false>
struct GridSource {
    static constexpr int kChunk = PIN_GRID_CHUNK;
    static constexpr int kSeg = kListSeg;
    static constexpr bool kIdPayload = IDP;
    const PinGrid& gr;
    const PinPoints& p;
    __device__ GridSource(const PinGrid& g_, const PinPoints& p_) : gr(g_), p(p_) {}

    // query cell relative to the box, clamped so that every offset stays representable in
    // int32 and a far-away query still lands outside the box for every offset
    __device__ __forceinline__ static int rel(float v, float r, int64_t o, int e) {
        const int64_t l = (int64_t)floorf(v / r) - o;
        return (int)(l < -256 ? -256 : (l > (int64_t)e + 256 ? (int64_t)e + 256 : l));
    }

    template <int CH>
    __device__ __forceinline__ int scan(float qx, float qy, float qz, TopK& tk) const {
#if defined(PIN_CHECK_SCAN) && PIN_CHECK_SCAN
        // self-check build (tools/check_scan.py): the brick-window scan -- its wave-major LDS
        // list shared with the decoder scratch -- against the per-cell scan, which uses no LDS;
        // the same cells in the same order must give the same count, payloads and distances
        // bitwise.  A mismatch poisons the query (nearest distance NaN -> NaN outputs).
        if (gr.window <= 2) {
            TopK t2;
            t2.init();
            const int n2 = scan_cells<CH>(qx, qy, qz, t2);
            const int n1 = scan_window<CH>(qx, qy, qz, tk);
            bool same = n1 == n2;
#pragma unroll
            for (int j = 0; j < kK; ++j)
                same = same && tk.g[j] == t2.g[j] && __float_as_int(tk.d[j]) == __float_as_int(t2.d[j]);
            if (!same) tk.d[0] = __int_as_float(0x7fc00000);
            return n1;
        }
#endif
        if (gr.window <= 2) return scan_window<CH>(qx, qy, qz, tk);
        return scan_cells<CH>(qx, qy, qz, tk);
    }

    // Brick-window scan (window <= 2): the 5x5x5-cell neighbourhood lies in <= 2 bricks per
    // axis, so the <= 8 bricks are loaded in ONE round trip; the occupied offsets (reference
    // cell order) are then found with register selects and their compact-record indices listed
    // in LDS (one column per lane: conflict-free, no barrier); records are fetched for listed
    // cells only, CH per round trip.
    template <int CH>
    __device__ __forceinline__ int scan_window(float qx, float qy, float qz, TopK& tk) const {
        int* const s_list = wave_list();
        const uint4* __restrict__ bricks = (const uint4*)gr.bricks;
        const float4* __restrict__ crec = (const float4*)gr.crec;
        const int32_t* __restrict__ offs = gr.offsets;
        const float res = gr.resolution, maxd2 = gr.max_valid_dist2;
        const int nbx = gr.dims.nbx, nby = gr.dims.nby, nbz = gr.dims.nbz;
        const int lx = rel(qx, res, gr.dims.ox, 4 * nbx);
        const int ly = rel(qy, res, gr.dims.oy, 4 * nby);
        const int lz = rel(qz, res, gr.dims.oz, 4 * nbz);
        const int bx0 = (lx - 2) >> 2, by0 = (ly - 2) >> 2, bz0 = (lz - 2) >> 2;
        uint32_t wl[8], wh[8], wp[8];
        {
            uint4 w[8];
            bool in[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int bx = bx0 + (k & 1), by = by0 + ((k >> 1) & 1), bz = bz0 + (k >> 2);
                in[k] = (unsigned)bx < (unsigned)nbx && (unsigned)by < (unsigned)nby && (unsigned)bz < (unsigned)nbz;
                w[k] = bricks[in[k] ? ((int64_t)bz * nby + by) * nbx + bx : 0];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                wl[k] = in[k] ? w[k].x : 0u;
                wh[k] = in[k] ? w[k].y : 0u;
                wp[k] = w[k].z;
            }
        }
        const int lane = threadIdx.x & 63;
        const int Kc = gr.num_cells;
        int nn = 0;
        if (gr.num_columns > 0) {
            // Column scan: per (x, y) column of the neighbourhood, the column's 4-bit z nibbles
            // of its two z-bricks give an 8-bit z-occupancy word; the column's cell run is a
            // shifted window of it, so empty cells cost nothing and only occupied cells are
            // ranked and listed (in the reference cell order: columns in order, z ascending).
            const int32_t* __restrict__ cols = offs + ((Kc + 15) & ~15);
            const int zr0 = lz - 4 * bz0;   // query z inside the 8-cell z span, 2..5
            int cnt = 0;
            for (int c = 0; c < gr.num_columns; ++c) {
                const int col = cols[c];
                const int nz = (col >> 24) & 255;
                if (__any(cnt + nz > kSeg)) {   // list full: consume it first (only for Kc > 32)
                    records_from_list<CH>(s_list, cnt, crec, qx, qy, qz, maxd2, tk, nn);
                    cnt = 0;
                }
                const int cx = lx + ((col & 255) - 128);
                const int cy = ly + (((col >> 8) & 255) - 128);
                const int kxy = ((cx >> 2) - bx0) | (((cy >> 2) - by0) << 1);
                const uint32_t lo0 = sel4v(wl[0], wl[1], wl[2], wl[3], kxy);
                const uint32_t hi0 = sel4v(wh[0], wh[1], wh[2], wh[3], kxy);
                const uint32_t lo1 = sel4v(wl[4], wl[5], wl[6], wl[7], kxy);
                const uint32_t hi1 = sel4v(wh[4], wh[5], wh[6], wh[7], kxy);
                const uint32_t pre0 = sel4v(wp[0], wp[1], wp[2], wp[3], kxy);
                const uint32_t pre1 = sel4v(wp[4], wp[5], wp[6], wp[7], kxy);
                const int sh = ((cx & 3) << 4) | ((cy & 3) << 2);
                const uint32_t n0 = (uint32_t)((((uint64_t)hi0 << 32) | lo0) >> sh) & 15u;
                const uint32_t n1 = (uint32_t)((((uint64_t)hi1 << 32) | lo1) >> sh) & 15u;
                const int zs = zr0 + (((col >> 16) & 255) - 128);
                uint32_t run = ((n0 | (n1 << 4)) >> zs) & ((1u << nz) - 1u);
                while (run) {
                    const int z = zs + __builtin_ctz(run);
                    run &= run - 1u;
                    const bool up = z >= 4;
                    const uint64_t bits = up ? (((uint64_t)hi1 << 32) | lo1) : (((uint64_t)hi0 << 32) | lo0);
                    const uint32_t pre = up ? pre1 : pre0;
                    const int bit = sh | (z & 3);
                    s_list[cnt * 64 + lane] = (int)(pre + (uint32_t)__popcll(bits & ((1ull << bit) - 1ull)));
                    ++cnt;
                }
            }
            records_from_list<CH>(s_list, cnt, crec, qx, qy, qz, maxd2, tk, nn);
            return nn;
        }
        for (int s0 = 0; s0 < Kc; s0 += kSeg) {
            const int s1 = Kc < s0 + kSeg ? Kc : s0 + kSeg;
            int cnt = 0;
            for (int t = s0; t < s1; ++t) {
                const int of = offs[t];
                const int cx = lx + ((of & 255) - 128);
                const int cy = ly + (((of >> 8) & 255) - 128);
                const int cz = lz + (((of >> 16) & 255) - 128);
                const int k = ((cx >> 2) - bx0) | (((cy >> 2) - by0) << 1) | (((cz >> 2) - bz0) << 2);
                const uint64_t bits = ((uint64_t)sel8(wh, k) << 32) | sel8(wl, k);
                const int bit = ((cx & 3) << 4) | ((cy & 3) << 2) | (cz & 3);
                if ((bits >> bit) & 1ull) {
                    s_list[cnt * 64 + lane] = (int)(sel8(wp, k) + (uint32_t)__popcll(bits & ((1ull << bit) - 1ull)));
                    ++cnt;
                }
            }
            records_from_list<CH>(s_list, cnt, crec, qx, qy, qz, maxd2, tk, nn);
        }
        return nn;
    }

    // Pair mode (small training batches, two lanes per query; ph = lane & 1): both lanes list the
    // same occupied cells, the even lane takes the first half of each list segment and the odd
    // lane the second, and the lists are merged in reference order at every segment flush (the
    // odd lane then restarts empty) and at the end.  Returns nn over both halves.  Outside the
    // column scan both lanes run the whole scan and the odd lane's result is dropped.
    template <int CH>
    __device__ __forceinline__ int scan_pair(float qx, float qy, float qz, TopK& tk, int ph) const {
        if (!(gr.window <= 2 && gr.num_columns > 0)) {
            int nn = scan<CH>(qx, qy, qz, tk);
            if (ph) {
                tk.init();
                nn = 0;
            }
            topk_pair_merge(tk, ph);
            return nn + __shfl_xor(nn, 1);
        }
        int* const s_list = wave_list();
        const uint4* __restrict__ bricks = (const uint4*)gr.bricks;
        const float4* __restrict__ crec = (const float4*)gr.crec;
        const int32_t* __restrict__ offs = gr.offsets;
        const float res = gr.resolution, maxd2 = gr.max_valid_dist2;
        const int nbx = gr.dims.nbx, nby = gr.dims.nby, nbz = gr.dims.nbz;
        const int lx = rel(qx, res, gr.dims.ox, 4 * nbx);
        const int ly = rel(qy, res, gr.dims.oy, 4 * nby);
        const int lz = rel(qz, res, gr.dims.oz, 4 * nbz);
        const int bx0 = (lx - 2) >> 2, by0 = (ly - 2) >> 2, bz0 = (lz - 2) >> 2;
        uint32_t wl[8], wh[8], wp[8];
        {
            uint4 w[8];
            bool in[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int bx = bx0 + (k & 1), by = by0 + ((k >> 1) & 1), bz = bz0 + (k >> 2);
                in[k] = (unsigned)bx < (unsigned)nbx && (unsigned)by < (unsigned)nby && (unsigned)bz < (unsigned)nbz;
                w[k] = bricks[in[k] ? ((int64_t)bz * nby + by) * nbx + bx : 0];
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                wl[k] = in[k] ? w[k].x : 0u;
                wh[k] = in[k] ? w[k].y : 0u;
                wp[k] = w[k].z;
            }
        }
        const int lane = threadIdx.x & 63;
        const int Kc = gr.num_cells;
        int nn = 0;
        const int32_t* __restrict__ cols = offs + ((Kc + 15) & ~15);
        const int zr0 = lz - 4 * bz0;
        int cnt = 0;
        for (int c = 0; c < gr.num_columns; ++c) {
            const int col = cols[c];
            const int nz = (col >> 24) & 255;
            if (__any(cnt + nz > kSeg)) {   // list full: its two halves, then the merge
                const int h = (cnt + 1) >> 1;
                records_from_range<CH>(s_list, ph ? h : 0, ph ? cnt : h, crec, qx, qy, qz, maxd2, tk, nn);
                topk_pair_merge(tk, ph);
                if (ph) tk.init();
                cnt = 0;
            }
            const int cx = lx + ((col & 255) - 128);
            const int cy = ly + (((col >> 8) & 255) - 128);
            const int kxy = ((cx >> 2) - bx0) | (((cy >> 2) - by0) << 1);
            const uint32_t lo0 = sel4v(wl[0], wl[1], wl[2], wl[3], kxy);
            const uint32_t hi0 = sel4v(wh[0], wh[1], wh[2], wh[3], kxy);
            const uint32_t lo1 = sel4v(wl[4], wl[5], wl[6], wl[7], kxy);
            const uint32_t hi1 = sel4v(wh[4], wh[5], wh[6], wh[7], kxy);
            const uint32_t pre0 = sel4v(wp[0], wp[1], wp[2], wp[3], kxy);
            const uint32_t pre1 = sel4v(wp[4], wp[5], wp[6], wp[7], kxy);
            const int sh = ((cx & 3) << 4) | ((cy & 3) << 2);
            const uint32_t n0 = (uint32_t)((((uint64_t)hi0 << 32) | lo0) >> sh) & 15u;
            const uint32_t n1 = (uint32_t)((((uint64_t)hi1 << 32) | lo1) >> sh) & 15u;
            const int zs = zr0 + (((col >> 16) & 255) - 128);
            uint32_t run = ((n0 | (n1 << 4)) >> zs) & ((1u << nz) - 1u);
            while (run) {
                const int z = zs + __builtin_ctz(run);
                run &= run - 1u;
                const bool up = z >= 4;
                const uint64_t bits = up ? (((uint64_t)hi1 << 32) | lo1) : (((uint64_t)hi0 << 32) | lo0);
                const uint32_t pre = up ? pre1 : pre0;
                const int bit = sh | (z & 3);
                s_list[cnt * 64 + lane] = (int)(pre + (uint32_t)__popcll(bits & ((1ull << bit) - 1ull)));
                ++cnt;
            }
        }
        const int h = (cnt + 1) >> 1;
        records_from_range<CH>(s_list, ph ? h : 0, ph ? cnt : h, crec, qx, qy, qz, maxd2, tk, nn);
        topk_pair_merge(tk, ph);
        return nn + __shfl_xor(nn, 1);
    }

    // Records of list entries [lo, hi) of the lane, CH per round trip (scan_pair)
    template <int CH>
    __device__ __forceinline__ static void records_from_range(const int* s_list, int lo, int hi,
                                                              const float4* __restrict__ crec, float qx, float qy,
                                                              float qz, float maxd2, TopK& tk, int& nn) {
        const int lane = threadIdx.x & 63;
        for (int j0 = lo; __any(j0 < hi); j0 += CH) {
            int ci[CH];
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int v = s_list[(j0 + u < kSeg ? j0 + u : kSeg - 1) * 64 + lane];   // stale slots are masked
                ci[u] = (j0 + u < hi) ? v : -1;
            }
            float4 r[CH];
#pragma unroll
            for (int u = 0; u < CH; ++u) r[u] = crec[ci[u] > 0 ? ci[u] : 0];
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int id = __float_as_int(r[u].w);
                const float d2 = dist2(r[u].x, r[u].y, r[u].z, qx, qy, qz);
                const bool ok = ci[u] >= 0 && id != -1 && d2 <= maxd2;
                nn += ok ? 1 : 0;
                tk.insert(ok ? d2 : INFINITY, IDP ? (id & kIdMask) : ci[u]);
            }
        }
    }

    // Records of the lane's listed candidates, CH gathers per round trip; the trip count is the
    // longest list among the ACTIVE lanes (__any ignores lanes that returned early in a partial
    // last wave).
    template <int CH>
    __device__ __forceinline__ static void records_from_list(const int* s_list, int cnt,
                                                             const float4* __restrict__ crec, float qx, float qy,
                                                             float qz, float maxd2, TopK& tk, int& nn) {
        const int lane = threadIdx.x & 63;
        for (int j0 = 0; __any(j0 < cnt); j0 += CH) {
            int ci[CH];
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int v = s_list[(j0 + u < kSeg ? j0 + u : kSeg - 1) * 64 + lane];   // stale slots are masked
                ci[u] = (j0 + u < cnt) ? v : -1;
            }
            float4 r[CH];
#pragma unroll
            for (int u = 0; u < CH; ++u) {
#if defined(PIN_PROF_STAGE) && PIN_PROF_STAGE == 5
                // profiling variant: records from an LDS table (wrong values; the payloads stay
                // valid compact indices, so later gathers stay in bounds): what a wave-staged
                // record set would cost
                __shared__ float4 s_fake[1024];
                r[u] = s_fake[(ci[u] > 0 ? ci[u] : 0) & 1023];
#else
                r[u] = crec[ci[u] > 0 ? ci[u] : 0];
#endif
            }
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int id = __float_as_int(r[u].w);
                const float d2 = dist2(r[u].x, r[u].y, r[u].z, qx, qy, qz);
                const bool ok = ci[u] >= 0 && id != -1 && d2 <= maxd2;
                nn += ok ? 1 : 0;
                tk.insert(ok ? d2 : INFINITY, IDP ? (id & kIdMask) : ci[u]);
            }
        }
    }

    // one cell of the reference's sort row (resolve_ties): cell c's candidate distance and
    // payload, 9e3 / -1 where the reference has idx -1 (c >= n: an unused entry)
    __device__ __forceinline__ int num_cells() const { return gr.num_cells; }
    __device__ __forceinline__ void ref_cell(float qx, float qy, float qz, int c, int n, float& k, int& g) const {
        const uint4* __restrict__ bricks = (const uint4*)gr.bricks;
        const float4* __restrict__ crec = (const float4*)gr.crec;
        const float res = gr.resolution, maxd2 = gr.max_valid_dist2;
        const int ex = 4 * gr.dims.nbx, ey = 4 * gr.dims.nby, ez = 4 * gr.dims.nbz;
        const int lx = rel(qx, res, gr.dims.ox, ex);
        const int ly = rel(qy, res, gr.dims.oy, ey);
        const int lz = rel(qz, res, gr.dims.oz, ez);
        const int of = gr.offsets[c < n ? c : 0];
        const int cx = lx + ((of & 255) - 128);
        const int cy = ly + (((of >> 8) & 255) - 128);
        const int cz = lz + (((of >> 16) & 255) - 128);
        const bool in = c < n && (unsigned)cx < (unsigned)ex && (unsigned)cy < (unsigned)ey && (unsigned)cz < (unsigned)ez;
        const uint4 w = bricks[in ? ((cz >> 2) * gr.dims.nby + (cy >> 2)) * gr.dims.nbx + (cx >> 2) : 0];
        const int bit = ((cx & 3) << 4) | ((cy & 3) << 2) | (cz & 3);
        const uint64_t bits = ((uint64_t)w.y << 32) | w.x;
        const bool set = in && ((bits >> bit) & 1ull);
        const int ci = set ? (int)(w.z + (uint32_t)__popcll(bits & ((1ull << bit) - 1ull))) : -1;
        const float4 v = crec[ci > 0 ? ci : 0];
        const int id = __float_as_int(v.w);
        const float d2 = dist2(v.x, v.y, v.z, qx, qy, qz);
        const bool ok = ci >= 0 && id != -1 && d2 <= maxd2;
        k = ok ? d2 : kInvalidDist2;
        g = ok ? (IDP ? (id & kIdMask) : ci) : -1;
    }

    // Per-cell scan (any window): CH cell lookups back to back, then CH record gathers.
    template <int CH>
    __device__ __forceinline__ int scan_cells(float qx, float qy, float qz, TopK& tk) const {
        const uint4* __restrict__ bricks = (const uint4*)gr.bricks;
        const float4* __restrict__ crec = (const float4*)gr.crec;
        const int32_t* __restrict__ offs = gr.offsets;  // padded to a multiple of 16 entries
        const float res = gr.resolution, maxd2 = gr.max_valid_dist2;
        const int ex = 4 * gr.dims.nbx, ey = 4 * gr.dims.nby, ez = 4 * gr.dims.nbz;
        const int lx = rel(qx, res, gr.dims.ox, ex);
        const int ly = rel(qy, res, gr.dims.oy, ey);
        const int lz = rel(qz, res, gr.dims.oz, ez);
        const int Kc = gr.num_cells;
        int nn = 0;
        for (int c0 = 0; c0 < Kc; c0 += CH) {
            int of[CH];
#pragma unroll
            for (int t = 0; t < CH; ++t) of[t] = offs[c0 + t];
            uint4 w[CH];
            int bit[CH];
            bool in[CH];
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const int cx = lx + ((of[t] & 255) - 128);
                const int cy = ly + (((of[t] >> 8) & 255) - 128);
                const int cz = lz + (((of[t] >> 16) & 255) - 128);
                in[t] = (c0 + t < Kc) && (unsigned)cx < (unsigned)ex && (unsigned)cy < (unsigned)ey &&
                        (unsigned)cz < (unsigned)ez;
                const int b = in[t] ? ((cz >> 2) * gr.dims.nby + (cy >> 2)) * gr.dims.nbx + (cx >> 2) : 0;
                bit[t] = ((cx & 3) << 4) | ((cy & 3) << 2) | (cz & 3);
                w[t] = bricks[b];
            }
            int ci[CH];
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const uint64_t bits = ((uint64_t)w[t].y << 32) | w[t].x;
                const bool set = in[t] && ((bits >> bit[t]) & 1ull);
                ci[t] = set ? (int)(w[t].z + (uint32_t)__popcll(bits & ((1ull << bit[t]) - 1ull))) : -1;
            }
            float4 r[CH];
#pragma unroll
            for (int t = 0; t < CH; ++t) r[t] = crec[ci[t] > 0 ? ci[t] : 0];
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const int id = __float_as_int(r[t].w);
                const float d2 = dist2(r[t].x, r[t].y, r[t].z, qx, qy, qz);
                const bool ok = ci[t] >= 0 && id != -1 && d2 <= maxd2;
                nn += ok ? 1 : 0;
                tk.insert(ok ? d2 : INFINITY, IDP ? (id & kIdMask) : ci[t]);
            }
        }
        return nn;
    }
    __device__ __forceinline__ float4 record(int pay) const {
        return ((const float4*)gr.crec)[pay > 0 ? pay : 0];
    }
    __device__ __forceinline__ void features(int pay, int64_t id, float4& f0, float4& f1) const {
        if (FAT) {
            const float4* r = (const float4*)gr.cfeat + 2 * (int64_t)(pay > 0 ? pay : 0);
            f0 = r[0];
            f1 = r[1];
        } else {
            const float4* __restrict__ feat = (const float4*)p.features;
            f0 = feat[2 * id];
            f1 = feat[2 * id + 1];
        }
    }
    __device__ __forceinline__ float certainty(int pay, int64_t id) const {
        if (FAT) return gr.ccert[pay > 0 ? pay : 0];
        return p.certainties[id];
    }
    __device__ __forceinline__ int gid(int pay) const { return pay >= 0 ? gr.cgid[pay] : -1; }
};

// passive quaternion rotation, utils/tools.py:316-323 (same op order)
__device__ __forceinline__ void quat_rotate_passive(float4 qt, float& vx, float& vy, float& vz) {
    const float ux = -qt.y, uy = -qt.z, uz = -qt.w, w = qt.x;
    const float tx = 2.f * (uy * vz - uz * vy);
    const float ty = 2.f * (uz * vx - ux * vz);
    const float tz = 2.f * (ux * vy - uy * vx);
    const float cx = uy * tz - uz * ty;
    const float cy = uz * tx - ux * tz;
    const float cz = ux * ty - uy * tx;
    vx = (vx + w * tx) + cx;
    vy = (vy + w * ty) + cy;
    vz = (vz + w * tz) + cz;
}

// active rotation matrix R(q) (w,x,y,z); the passive rotation of tools.py:316 is R(q)^T v
__device__ __forceinline__ void quat_rotmat(float4 qt, float (&R)[3][3]) {
    const float w = qt.x, x = qt.y, y = qt.z, z = qt.w;
    R[0][0] = 1.f - 2.f * (y * y + z * z); R[0][1] = 2.f * (x * y - w * z); R[0][2] = 2.f * (x * z + w * y);
    R[1][0] = 2.f * (x * y + w * z); R[1][1] = 1.f - 2.f * (x * x + z * z); R[1][2] = 2.f * (y * z - w * x);
    R[2][0] = 2.f * (x * z - w * y); R[2][1] = 2.f * (y * z + w * x); R[2][2] = 1.f - 2.f * (x * x + y * y);
}

// R(q) g: transpose of the passive rotation's Jacobian applied to g (d vec/dq = R(q)^T)
__device__ __forceinline__ void quat_rotate_active(float4 qt, float gx, float gy, float gz, float& ox, float& oy,
                                                   float& oz) {
    const float w = qt.x, x = qt.y, y = qt.z, z = qt.w;
    ox = (1.f - 2.f * (y * y + z * z)) * gx + 2.f * (x * y - w * z) * gy + 2.f * (x * z + w * y) * gz;
    oy = 2.f * (x * y + w * z) * gx + (1.f - 2.f * (x * x + z * z)) * gy + 2.f * (y * z - w * x) * gz;
    oz = 2.f * (x * z - w * y) * gx + 2.f * (y * z + w * x) * gy + (1.f - 2.f * (x * x + y * y)) * gz;
}

// Neighbour set of one query after the scan (weights, distance terms, neighbour vectors;
// feature rows are gathered by gather_inputs when needed so they do not stay live).
struct Neighbours {
    float w[kK];      // normalised IDW weights (0 for invalid)
    float u[kK];      // un-normalised 1/(d2+eps) (0 for invalid)
    float S;          // sum of u
    float pg[kK][3];  // q - global position (drives the distance gradient)
    float v[kK][3];   // q - local position (decoder input before the optional rotation)
    int id[kK];       // feature row, -1 invalid
    int pay[kK];      // source payload of the candidate (global index or compact record)
};

// neural_points.py:618-632 on the top-k: u = 1/(d2+eps), S = sum u, w = u/S (0 when invalid).
// All record gathers are unconditional; the rare "unfaithful" records (local position !=
// global one, the global2local quirk) take a wave-uniform branch for their extra gather.
template <class Src>
__device__ __forceinline__ void load_topk(const Src& src, const PinPoints& p, const TopK& tk, int nn, int nn_k,
                                          float qx, float qy, float qz, Neighbours& nb) {
    float4 r[kK];
#pragma unroll
    for (int j = 0; j < kK; ++j) r[j] = src.record(tk.g[j]);
    float S = 0.f;
    bool unf = false;
#pragma unroll
    for (int j = 0; j < kK; ++j) {
        const int raw = __float_as_int(r[j].w);
        const bool valid = j < nn_k && tk.g[j] >= 0;
        nb.id[j] = valid ? (raw & kIdMask) : -1;
        nb.pay[j] = valid ? tk.g[j] : -1;
        unf |= valid && (raw & PIN_RECORD_UNFAITHFUL);
        nb.u[j] = valid ? 1.0f / (tk.d[j] + kIdwEps) : 0.f;
        S = S + nb.u[j];
        nb.pg[j][0] = qx - r[j].x;
        nb.pg[j][1] = qy - r[j].y;
        nb.pg[j][2] = qz - r[j].z;
        nb.v[j][0] = nb.pg[j][0];
        nb.v[j][1] = nb.pg[j][1];
        nb.v[j][2] = nb.pg[j][2];
    }
    nb.S = S;
#pragma unroll
    for (int j = 0; j < kK; ++j) nb.w[j] = (nb.id[j] >= 0 && nn > 0) ? nb.u[j] / S : 0.f;
    if (__any(unf)) {
#pragma unroll
        for (int j = 0; j < kK; ++j) {
            const int raw = __float_as_int(r[j].w);
            if (nb.id[j] >= 0 && (raw & PIN_RECORD_UNFAITHFUL)) {
                const int64_t id = nb.id[j];
                nb.v[j][0] = qx - p.positions[3 * id];
                nb.v[j][1] = qy - p.positions[3 * id + 1];
                nb.v[j][2] = qz - p.positions[3 * id + 2];
            }
        }
    }
}

// Decoder inputs of neighbours [J0, J0+NJ): feature rows (2 x 16 B each) and neighbour
// vectors, passively rotated by the point quaternion after pgo (neural_points.py:577-614).
// Gathers are unconditional (invalid neighbours read row 0) and zeroed afterwards.
template <bool PGO, int J0, int NJ, class Src>
__device__ __forceinline__ void gather_inputs(const Src& src, const PinPoints& p, const Neighbours& nb,
                                              float (&x)[NJ][kD], float4 (&quat)[NJ]) {
#pragma unroll
    for (int t = 0; t < NJ; ++t) {
        const int j = J0 + t;
        const int64_t id = nb.id[j] > 0 ? nb.id[j] : 0;
        float4 f0, f1;
        src.features(nb.pay[j], id, f0, f1);
        x[t][0] = f0.x; x[t][1] = f0.y; x[t][2] = f0.z; x[t][3] = f0.w;
        x[t][4] = f1.x; x[t][5] = f1.y; x[t][6] = f1.z; x[t][7] = f1.w;
        x[t][8] = nb.v[j][0];
        x[t][9] = nb.v[j][1];
        x[t][10] = nb.v[j][2];
        quat[t] = make_float4(1.f, 0.f, 0.f, 0.f);
        if (PGO) quat[t] = ((const float4*)p.orientations)[id];
    }
#pragma unroll
    for (int t = 0; t < NJ; ++t) {
        const bool valid = nb.id[J0 + t] >= 0;
        if (PGO) quat_rotate_passive(quat[t], x[t][8], x[t][9], x[t][10]);
#pragma unroll
        for (int d = 0; d < kD; ++d) x[t][d] = valid ? x[t][d] : 0.f;
    }
}

// sum_j cert_j * w_j with unconditional gathers (neural_points.py:651-656)
template <class Src>
__device__ __forceinline__ float gather_certainty(const Src& src, const Neighbours& nb) {
    float c[kK];
#pragma unroll
    for (int j = 0; j < kK; ++j) c[j] = src.certainty(nb.pay[j], nb.id[j] > 0 ? nb.id[j] : 0);
    float cert = 0.f;
#pragma unroll
    for (int j = 0; j < kK; ++j) cert = cert + (nb.id[j] >= 0 ? c[j] : 0.f) * nb.w[j];
    return cert;
}

// Decoder weights staged in LDS once per block (stage_mlp), laid out for the packed loop:
// hidden units in pairs (c, c+1), W1 interleaved per input i as {W1[c][i], W1[c+1][i]}
// (12 inputs incl. one pad -> 24 floats per pair), then b1, W2, b2.  A pair's operand for
// v_pk_fma_f32 is one 8-B broadcast LDS read; broadcast reads return in order, so several
// stay in flight (the scalar-load form paid a dependent K$ round trip per pair).
constexpr int kWRow = 12;                    // padded inputs per hidden unit
constexpr int kWPair = 2 * kWRow;            // floats per hidden-unit pair
constexpr int kWB1 = kH * kWRow;
constexpr int kWW2 = kWB1 + kH;
constexpr int kWB2 = kWW2 + kH;
constexpr int kWSize = kWB2 + 4;

struct MlpW {
    const float* w;   // LDS
    float sdf_scale;
    float* xs;        // per-wave LDS scratch of the MFMA decoders, or nullptr
    const unsigned char* pk = nullptr;   // LDS copy of the pin_mlp_pack image (mlp_sdf_mfma16)
};

#ifndef PIN_MLP_ROWS
#define PIN_MLP_ROWS 0   // 1: W1 staged row-major and decoded one hidden unit at a time (mlp_sdf_rows)
#endif

// W1[c][i] in the staged layout
__device__ __forceinline__ int w1_at(int c, int i) {
    return PIN_MLP_ROWS ? c * kWRow + i : (c >> 1) * kWPair + 2 * i + (c & 1);
}

// all threads of the block must call this (it ends with a barrier)
__device__ __forceinline__ MlpW stage_mlp(const PinMlp& m, float* s_w) {
    for (int e = threadIdx.x; e < kWSize; e += blockDim.x) {
        float v = 0.f;
        if (e < kWB1) {
            int c, i;
            if (PIN_MLP_ROWS) {
                c = e / kWRow;
                i = e - c * kWRow;
            } else {
                const int pr = e / kWPair, r = e - pr * kWPair;
                i = r >> 1;
                c = 2 * pr + (r & 1);
            }
            v = i < kD ? m.W1[c * kD + i] : 0.f;
        } else if (e < kWW2) {
            v = m.b1[e - kWB1];
        } else if (e < kWB2) {
            v = m.W2[e - kWW2];
        } else if (e == kWB2) {
            v = m.b2[0];
        }
        s_w[e] = v;
    }
    __syncthreads();
    return MlpW{s_w, m.sdf_scale, nullptr};
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

// row c of W1 from the staged layout (stride-2 reads)
__device__ __forceinline__ void load_row(const float* __restrict__ w, int c, float (&r)[kWRow]) {
#pragma unroll
    for (int i = 0; i < kWRow; ++i) r[i] = w[w1_at(c, i)];
}

// Decoder forward fused with its input gradient (model/decoder.py:66-88):
//   sdf = s * (w2 . relu(W1 x + b1) + b2),  gx[i] = s * sum_c w2[c] 1[pre_c > 0] W1[c][OFF+i].
// One pass over the hidden units, two at a time with packed FMAs (v_pk_fma_f32).
// mask (may be NULL): the 64 ReLU masks, bit c = [pre_c > 0] (the per-neighbour training forward
// saves them for the backward's input gradient, mlp_grad8_from_mask).
template <bool GRAD, int OFF, int NOUT>
__device__ __forceinline__ float mlp_sdf_packed(const MlpW& m, const float (&x)[kD], float (&gx)[NOUT],
                                                uint64_t* mask = nullptr) {
    f32x2 out2 = {0.f, 0.f};
    uint64_t mk = 0;
    f32x2 g2[NOUT];
#pragma unroll
    for (int i = 0; i < NOUT; ++i) g2[i] = (f32x2){0.f, 0.f};
#pragma unroll PIN_MLP_UNROLL
    for (int c = 0; c < kH; c += 2) {
        const f32x2* __restrict__ wp = (const f32x2*)(m.w + (c >> 1) * kWPair);
        f32x2 wv[kD];
#pragma unroll
        for (int i = 0; i < kD; ++i) wv[i] = wp[i];
        const f32x2 b = *(const f32x2*)(m.w + kWB1 + c);
        const f32x2 v2 = *(const f32x2*)(m.w + kWW2 + c);
        f32x2 acc = {0.f, 0.f};
#pragma unroll
        for (int i = 0; i < kD; ++i) acc = __builtin_elementwise_fma(wv[i], (f32x2){x[i], x[i]}, acc);
        const f32x2 pre = acc + b;
        const f32x2 a = {pre.x > 0.f ? v2.x : 0.f, pre.y > 0.f ? v2.y : 0.f};
        out2 = __builtin_elementwise_fma(a, pre, out2);
        if (mask) mk |= (uint64_t)((pre.x > 0.f ? 1u : 0u) | (pre.y > 0.f ? 2u : 0u)) << c;
        if (GRAD) {
#pragma unroll
            for (int i = 0; i < NOUT; ++i) g2[i] = __builtin_elementwise_fma(a, wv[OFF + i], g2[i]);
        }
    }
    if (GRAD) {
#pragma unroll
        for (int i = 0; i < NOUT; ++i) gx[i] = (g2[i].x + g2[i].y) * m.sdf_scale;
    }
    if (mask) *mask = mk;
    return ((out2.x + out2.y) + m.w[kWB2]) * m.sdf_scale;
}

// Two decodes sharing the weight reads (SDF and ReLU masks only, no gradient): the per-neighbour
// training forward decodes neighbours j and j + 1 of a row together -- one LDS broadcast read of a
// hidden-unit pair feeds both rows' packed FMAs, and the two chains are independent.  Each result
// is mlp_sdf_packed<false>'s, bitwise (the same operations in the same order per row).
__device__ __forceinline__ void mlp_sdf_packed_x2(const MlpW& m, const float (&xa)[kD], const float (&xb)[kD],
                                                  float& sa, float& sb, uint64_t& mka, uint64_t& mkb) {
    f32x2 oa = {0.f, 0.f}, ob = {0.f, 0.f};
    uint64_t ka = 0, kb = 0;
#pragma unroll PIN_MLP_UNROLL
    for (int c = 0; c < kH; c += 2) {
        const f32x2* __restrict__ wp = (const f32x2*)(m.w + (c >> 1) * kWPair);
        f32x2 wv[kD];
#pragma unroll
        for (int i = 0; i < kD; ++i) wv[i] = wp[i];
        const f32x2 b = *(const f32x2*)(m.w + kWB1 + c);
        const f32x2 v2 = *(const f32x2*)(m.w + kWW2 + c);
        f32x2 acca = {0.f, 0.f}, accb = {0.f, 0.f};
#pragma unroll
        for (int i = 0; i < kD; ++i) {
            acca = __builtin_elementwise_fma(wv[i], (f32x2){xa[i], xa[i]}, acca);
            accb = __builtin_elementwise_fma(wv[i], (f32x2){xb[i], xb[i]}, accb);
        }
        const f32x2 pa = acca + b, pb = accb + b;
        const f32x2 aa = {pa.x > 0.f ? v2.x : 0.f, pa.y > 0.f ? v2.y : 0.f};
        const f32x2 ab = {pb.x > 0.f ? v2.x : 0.f, pb.y > 0.f ? v2.y : 0.f};
        oa = __builtin_elementwise_fma(aa, pa, oa);
        ob = __builtin_elementwise_fma(ab, pb, ob);
        ka |= (uint64_t)((pa.x > 0.f ? 1u : 0u) | (pa.y > 0.f ? 2u : 0u)) << c;
        kb |= (uint64_t)((pb.x > 0.f ? 1u : 0u) | (pb.y > 0.f ? 2u : 0u)) << c;
    }
    sa = ((oa.x + oa.y) + m.w[kWB2]) * m.sdf_scale;
    sb = ((ob.x + ob.y) + m.w[kWB2]) * m.sdf_scale;
    mka = ka;
    mkb = kb;
}

// The same decoder one hidden unit at a time with plain FMAs (v_fma_f32 issues in 2 cycles per
// wave64 on a SIMD-32, so packing buys no FLOP rate on gfx950): the W1 row comes from LDS as
// three 16-B broadcast reads, and only x, the gradient accumulators and one row are live --
// about 40 VGPRs instead of the packed form's ~90, which is what lets the fused SDF+gradient
// kernel fit 128 VGPRs (4 waves per SIMD).
template <bool GRAD, int OFF, int NOUT>
__device__ __forceinline__ float mlp_sdf_rows(const MlpW& m, const float (&x)[kD], float (&gx)[NOUT]) {
    float out = 0.f;
    float g[NOUT];
#pragma unroll
    for (int i = 0; i < NOUT; ++i) g[i] = 0.f;
#pragma unroll PIN_MLP_UNROLL
    for (int c = 0; c < kH; ++c) {
        const float* __restrict__ wr = m.w + c * kWRow;   // row-major staging (PIN_MLP_ROWS)
        const float4 w0 = *(const float4*)(wr), w1 = *(const float4*)(wr + 4), w2 = *(const float4*)(wr + 8);
        const float w[kWRow] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w, w2.x, w2.y, w2.z, w2.w};
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < kD; ++i) acc = fmaf(w[i], x[i], acc);
        const float pre = acc + m.w[kWB1 + c];
        const float a = pre > 0.f ? m.w[kWW2 + c] : 0.f;
        out = fmaf(a, pre, out);
        if (GRAD) {
#pragma unroll
            for (int i = 0; i < NOUT; ++i) g[i] = fmaf(a, w[OFF + i], g[i]);
        }
    }
    if (GRAD) {
#pragma unroll
        for (int i = 0; i < NOUT; ++i) gx[i] = g[i] * m.sdf_scale;
    }
    return (out + m.w[kWB2]) * m.sdf_scale;
}

template <bool GRAD, int OFF, int NOUT>
__device__ __forceinline__ float mlp_sdf(const MlpW& m, const float (&x)[kD], float (&gx)[NOUT],
                                         uint64_t* mask = nullptr) {
    if constexpr (PIN_MLP_ROWS != 0) return mlp_sdf_rows<GRAD, OFF, NOUT>(m, x, gx);   // experiment: no masks
    else return mlp_sdf_packed<GRAD, OFF, NOUT>(m, x, gx, mask);
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// LDS ordering between lanes of one wave (a wave's DS instructions execute in order; this keeps
// the compiler from moving them across the exchange point)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The decoder of the wave's 64 queries as one batched GEMM on the f32 MFMA
// (v_mfma_f32_16x16x4_f32, exact f32 products; model/decoder.py:66-88):
//   P^T = W1 X^T             M = 64 hidden (4 tiles), N = 64 queries (4 tiles), K = 11 -> 12
//   sdf = s (w2 . relu(P + b1) + b2)    relu and the w2 dot on the accumulator tiles
//   gx^T = W1^T G^T,  G = w2 o 1[P + b1 > 0]    the masked tile is the next MFMA's B operand as
//                     it stands (K-step s pairs hidden unit 16mt + 4k + s with lane group k)
// X goes through 3 KB of LDS (xs) to reach the B-operand layout, and gx back through it.
// gx: the NOUT input gradients from input OFF on (OFF 0 / 11 weighted_first, OFF 8 / 3 for the
// neighbour-vector gradient of per-neighbour decoding).  Every lane of the wave must call this
// (lanes without a query pass zeros).
template <bool GRAD, int OFF, int NOUT>
__device__ __forceinline__ float mlp_sdf_wave(const MlpW& m, const float (&x)[kD], float (&gx)[NOUT]) {
    float* xs = m.xs;
    const int lane = threadIdx.x & 63;
    const int col = lane & 15, grp = lane >> 4;
    float4* xr = (float4*)(xs + lane * kWRow);
    xr[0] = make_float4(x[0], x[1], x[2], x[3]);
    xr[1] = make_float4(x[4], x[5], x[6], x[7]);
    xr[2] = make_float4(x[8], x[9], x[10], 0.f);
    wave_lds_sync();
    float bq[4][3];   // B[k = grp][j = col] = X[q = 16 nt + col][i = 4 ks + grp]
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) bq[nt][ks] = xs[(16 * nt + col) * kWRow + 4 * ks + grp];
    float outp[4] = {0.f, 0.f, 0.f, 0.f};
    f32x4 gacc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) gacc[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int mt = 0; mt < 4; ++mt) {
        float a[3];       // A[i = col -> hidden 16 mt + col][k = grp -> input 4 ks + grp]
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) a[ks] = m.w[w1_at(16 * mt + col, 4 * ks + grp)];   // input 11 is the 0 pad
        float b1v[4], w2v[4], ga[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int c = 16 * mt + 4 * grp + r;   // hidden unit of accumulator row r
            b1v[r] = m.w[kWB1 + c];
            w2v[r] = m.w[kWW2 + c];
            ga[r] = (GRAD && col < NOUT) ? m.w[w1_at(c, OFF + col)] : 0.f;   // A[i = col][k = grp] = W1[c][OFF+col]
        }
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            f32x4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 3; ++ks) d = __builtin_amdgcn_mfma_f32_16x16x4f32(a[ks], bq[nt][ks], d, 0, 0, 0);
            float g[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float pre = d[r] + b1v[r];
                const bool on = pre > 0.f;
                outp[nt] = on ? fmaf(w2v[r], pre, outp[nt]) : outp[nt];
                g[r] = on ? w2v[r] : 0.f;
            }
            if (GRAD) {
#pragma unroll
                for (int r = 0; r < 4; ++r) gacc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(ga[r], g[r], gacc[nt], 0, 0, 0);
            }
        }
    }
    // w2 . relu: sum the four lane groups of each query column; lane q keeps column q
    float out = 0.f;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        float v = outp[nt];
        v += __shfl_xor(v, 16);
        v += __shfl_xor(v, 32);
        out = (grp == nt) ? v : out;
    }
    if (GRAD) {
        wave_lds_sync();   // every lane has read its B operands
        if (4 * grp < NOUT) {     // rows i = 4 grp + r < 12 hold outputs
#pragma unroll
            for (int nt = 0; nt < 4; ++nt)
                *(float4*)(xs + (16 * nt + col) * kWRow + 4 * grp) =
                    make_float4(gacc[nt][0], gacc[nt][1], gacc[nt][2], gacc[nt][3]);
        }
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < NOUT; ++i) gx[i] = xs[lane * kWRow + i] * m.sdf_scale;
        wave_lds_sync();   // the next call's X staging reuses xs
    }
    return (out + m.w[kWB2]) * m.sdf_scale;
}

// ------------------------------------------------------------------ f16 matrix-core decoder
// The wave's 64 decodes as two GEMMs on v_mfma_f32_16x16x32_f16 with every f32 operand split
// into two f16 terms (pin_mlp_pack, include/pin_slam_amd.h):
//   GEMM1  P^T[c][q]  = sum_k A1[c][k] B1[k][q]        K-slots: Wh.xh | Wl.xh | b1h.E b1l.E (16x16x32)
//                                                      + Wh.xl (a second 16x16x32, K-slots 11..31 zero;
//                                                      a 16x16x16 chained onto the 16x16x32 accumulator
//                                                      measured wrong sums in tools/mf_unit.hip)
//   GEMM2  g^T[i][q]  = sum_c A2[i][c] 1[P[c][q] > 0]  A2 = (W1 o w2)^T split hi/lo, row 11 = w2 o b1
//   sdf = s (x . g + g_11 + b2),  dsdf/dx_i = s g_i
// B1 column q is query q's inputs scaled by E = 2^e_q (max|x| to [2^13, 2^14)), so D1 = 2^(e_c+e_q)
// P and only its sign is used; the GEMM2 B operand is the 0/1 mask, exact in f16, taken from
// the GEMM1 accumulators as they stand (K-slot s of lane group g <-> hidden 4g+s / 16+4g+s-4).
// Per lane: ~55 VALU for the split, 64 x 2.5 for the masks, ~40 to read g back -- against
// ~830 packed-FMA instructions for the VALU decoder -- and 48 MFMAs per wave.
constexpr int kPkA1 = 0;                    // [4 mt][64 lanes] f16x8   GEMM1 K-slots 8g..8g+7
constexpr int kPkA2 = kPkA1 + 4 * 64 * 16;  // [2 ch][2 term][64 lanes] f16x8
constexpr int kPkScale = kPkA2 + 4 * 64 * 16;   // [16] f32: 2^-f_i of GEMM2 row i
constexpr int kPkB2 = kPkScale + 16 * 4;        // f32 b2
constexpr int kPkBytes = 8288;

// ------------------------------------------------------------------ decoder pack (pin_mlp_pack)
// power of two taking max|row| to [2^13, 2^14) (any power for an all-zero row)
__device__ __forceinline__ float pack_row_scale(float mx) {
    const int eb = (__float_as_int(mx) >> 23) & 0xff;
    const int e = min(max(140 - eb, -100), 100);
    return __int_as_float((e + 127) << 23);
}

__device__ __forceinline__ void pack_split_f16(float v, int part, _Float16* out) {
    const _Float16 h = (_Float16)v;
    *out = part == 0 ? h : (_Float16)(v - (float)h);
}

// pin_mlp_pack's image, written by one block of 256 threads (k_mlp_pack; the training Adam step's
// decoder block right after it steps the parameters)
__device__ __forceinline__ void mlp_pack_block(const PinMlp& m, unsigned char* __restrict__ out) {
    __shared__ float s_e1[kH];          // GEMM1 row scales 2^e_c
    __shared__ float s_f[16];           // GEMM2 row scales 2^f_i
    __shared__ float s_a2[12][kH];      // GEMM2 rows: W1[c][i] w2[c] (i < 11), w2[c] b1[c] (i = 11)
    const int t = threadIdx.x;
    if (t < kH) {
        float mx = fabsf(m.b1[t]);
        for (int i = 0; i < kD; ++i) mx = fmaxf(mx, fabsf(m.W1[t * kD + i]));
        s_e1[t] = pack_row_scale(mx);
    }
    for (int e = t; e < 12 * kH; e += 256) {
        const int i = e / kH, c = e - i * kH;
        s_a2[i][c] = i < kD ? m.W1[c * kD + i] * m.W2[c] : m.W2[c] * m.b1[c];
    }
    __syncthreads();
    if (t < 16) {
        float mx = 0.f;
        if (t < 12)
            for (int c = 0; c < kH; ++c) mx = fmaxf(mx, fabsf(s_a2[t][c]));
        const float f = pack_row_scale(mx);
        s_f[t] = f;
        ((float*)(out + kPkScale))[t] = 1.f / f;   // exact: a power of two
    }
    if (t == 0) *(float*)(out + kPkB2) = m.b2[0];
    __syncthreads();
    // GEMM1 A: row c = 16 mt + lane % 16, K-slot k = 8 (lane / 16) + s:
    //   k < 11 W1 hi, k < 22 W1[k-11] lo, 22 b1 hi, 23 b1 lo, else 0 (B: x hi, x hi, E, E, -)
    for (int e = t; e < 4 * 64 * 8; e += 256) {
        const int mt = e >> 9, lane = (e >> 3) & 63, k = 8 * (lane >> 4) + (e & 7);
        const int c = 16 * mt + (lane & 15);
        const float sc = s_e1[c];
        _Float16* o = (_Float16*)(out + kPkA1) + e;
        if (k < 11) pack_split_f16(m.W1[c * kD + k] * sc, 0, o);
        else if (k < 22) pack_split_f16(m.W1[c * kD + k - 11] * sc, 1, o);
        else if (k < 24) pack_split_f16(m.b1[c] * sc, k - 22, o);
        else *o = (_Float16)0.f;
    }
    // GEMM2 A: [ch][term][lane] row i = lane % 16, slot s <-> hidden 32 ch + (s < 4 ? 4g + s : 16 + 4g + s - 4)
    for (int e = t; e < 2 * 2 * 64 * 8; e += 256) {
        const int ch = e >> 10, term = (e >> 9) & 1, lane = (e >> 3) & 63, sl = e & 7, g = lane >> 4;
        const int i = lane & 15;
        const int c = 32 * ch + (sl < 4 ? 4 * g + sl : 16 + 4 * g + sl - 4);
        _Float16* o = (_Float16*)(out + kPkA2) + e;
        if (i < 12) pack_split_f16(s_a2[i][c] * s_f[i], term, o);
        else *o = (_Float16)0.f;
    }
}
static_assert(kPkB2 + 4 <= kPkBytes && kPkBytes == PIN_MLP_PACK_BYTES && kPkBytes % 16 == 0, "pack layout");
#ifndef PIN_MF_NT_OUTER
#define PIN_MF_NT_OUTER 0   // 1: query tile as the outer GEMM loop (fewer live VGPRs, A re-read per tile)
#endif
constexpr int kXsStride = 20;               // floats per query row of the decoder scratch (80 B: conflict-free)
constexpr int kXsWave = 64 * kXsStride;     // floats of scratch per wave

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pack_f16x2(float a, float b) {
    return __builtin_bit_cast(uint32_t, (f16x2){(_Float16)a, (_Float16)b});
}

// 1.0h in each half whose accumulator is > 0 (relu' with torch's convention at 0 and NaN)
__device__ __forceinline__ uint32_t mask_f16x2(float a, float b) {
    return (a > 0.f ? 0x3C00u : 0u) | (b > 0.f ? 0x3C000000u : 0u);
}

// All 64 lanes of the wave must call this together (lanes without a query pass zeros).
// Returns sdf; gx = the NOUT input gradients from input OFF on (GRAD); mask (may be NULL): the
// lane's query's 64 ReLU masks, bit c = [pre_c > 0] (the decoder-parameter products of the
// training backward).
// NT: the query tile as the outer GEMM loop (fewer live VGPRs, the A tiles re-read from LDS per
// tile): slower where the kernel fits its register budget anyway, faster where it would spill
// (the weighted-first after-PGO query, compiled for 2 waves/SIMD: 97 -> 70 us per 262K step).
template <bool GRAD, int OFF, int NOUT, bool NT = (PIN_MF_NT_OUTER != 0)>
__device__ __forceinline__ float mlp_sdf_mfma16(const MlpW& m, const float (&x)[kD], float (&gx)[NOUT],
                                                uint64_t* mask = nullptr) {
    static_assert(OFF + NOUT <= kD, "decoder input range");
    float* xs = m.xs;
    const unsigned char* pk = m.pk;
    const int lane = threadIdx.x & 63;
    const int col = lane & 15, grp = lane >> 4;
    wave_lds_sync();   // xs aliases the wave's scan list: every lane is past its scan reads
    // ---- this lane's query as B1 column: scale, split, one 80-B LDS row
    float mx = 0.f;
#pragma unroll
    for (int i = 0; i < kD; ++i) mx = fmaxf(mx, fabsf(x[i]));
    const int eb = (__float_as_int(mx) >> 23) & 0xff;
    const int e = min(max(140 - eb, -14), 15);            // 2^e a normal f16
    const float sc = __int_as_float((e + 127) << 23);
    float xh[kD], xl[kD];
#pragma unroll
    for (int i = 0; i < kD; ++i) {
        const float v = x[i] * sc;
        xh[i] = __int_as_float(__float_as_int(v) & (int)0xFFFFE000u);   // 11 significant bits: exact f16
        xl[i] = v - xh[i];
    }
    {
        uint4* row = (uint4*)(xs + lane * kXsStride);
        row[0] = make_uint4(pack_f16x2(xh[0], xh[1]), pack_f16x2(xh[2], xh[3]), pack_f16x2(xh[4], xh[5]),
                            pack_f16x2(xh[6], xh[7]));
        row[1] = make_uint4(pack_f16x2(xh[8], xh[9]), pack_f16x2(xh[10], xh[0]), pack_f16x2(xh[1], xh[2]),
                            pack_f16x2(xh[3], xh[4]));
        row[2] = make_uint4(pack_f16x2(xh[5], xh[6]), pack_f16x2(xh[7], xh[8]), pack_f16x2(xh[9], xh[10]),
                            pack_f16x2(sc, sc));
        row[3] = make_uint4(pack_f16x2(xl[0], xl[1]), pack_f16x2(xl[2], xl[3]), pack_f16x2(xl[4], xl[5]),
                            pack_f16x2(xl[6], xl[7]));
        row[4] = make_uint4(pack_f16x2(xl[8], xl[9]), pack_f16x2(xl[10], 0.f), 0u, 0u);
    }
    wave_lds_sync();
    // B operands of the four query tiles (lane group 3 reads lo-row halves; its A slots are 0)
    uint32_t mbits[4][2] = {{0u, 0u}, {0u, 0u}, {0u, 0u}, {0u, 0u}};   // ReLU masks: [query tile][hidden half]
    if constexpr (NT) {
    // query tile outer: one tile's B operands, masks and GEMM2 accumulator live at a time (the A
    // tiles are re-read from LDS per tile); g of tile nt is written over its own, consumed B rows
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const float* rb = xs + (16 * nt + col) * kXsStride;
        const f16x8 bh = *(const f16x8*)(rb + 4 * grp);
        const f16x8 bl = *(const f16x8*)(rb + 12 + 4 * min(grp, 1));
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ch = 0; ch < 2; ++ch) {
            uint32_t mk[4];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int mt = 2 * ch + h;
                const f16x8 a = ((const f16x8*)(pk + kPkA1))[mt * 64 + lane];
                const uint4 au = __builtin_bit_cast(uint4, a);
                const f16x8 al = __builtin_bit_cast(
                    f16x8, make_uint4(grp < 2 ? au.x : 0u, grp == 0 ? au.y : (grp == 1 ? (au.y & 0xFFFFu) : 0u),
                                      grp == 0 ? au.z : 0u, grp == 0 ? au.w : 0u));
                f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bh, (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                d = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bl, d, 0, 0, 0);
                mk[2 * h] = mask_f16x2(d[0], d[1]);
                mk[2 * h + 1] = mask_f16x2(d[2], d[3]);
                if (mask) {   // as in the default order below
                    const uint32_t b4 = (d[0] > 0.f ? 1u : 0u) | (d[1] > 0.f ? 2u : 0u) | (d[2] > 0.f ? 4u : 0u) |
                                        (d[3] > 0.f ? 8u : 0u);
                    mbits[nt][ch] |= b4 << (16 * h + 4 * grp);
                }
            }
            const f16x8 a2h = ((const f16x8*)(pk + kPkA2))[(2 * ch) * 64 + lane];
            const f16x8 a2l = ((const f16x8*)(pk + kPkA2))[(2 * ch + 1) * 64 + lane];
            const f16x8 b = __builtin_bit_cast(f16x8, make_uint4(mk[0], mk[1], mk[2], mk[3]));
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2h, b, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2l, b, acc, 0, 0, 0);
        }
        wave_lds_sync();   // every lane has read tile nt's B rows
        if (grp < 3) *(f32x4*)(xs + (16 * nt + col) * kXsStride + 4 * grp) = acc;
    }
    wave_lds_sync();
    } else {
    f16x8 bh[4];
    f16x8 bl[4];   // x-lo rows: groups 2, 3 re-read group 1's slots (their A slots are 0)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const float* r = xs + (16 * nt + col) * kXsStride;
        bh[nt] = *(const f16x8*)(r + 4 * grp);
        bl[nt] = *(const f16x8*)(r + 12 + 4 * min(grp, 1));
    }
    f32x4 acc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
        uint32_t mk[4][4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int mt = 2 * ch + h;
            const f16x8 a = ((const f16x8*)(pk + kPkA1))[mt * 64 + lane];
            // Wh.xl: its K-slots 0..10 are A1's own slots 0..10 (lane groups 0 and 1), the rest 0
            const uint4 au = __builtin_bit_cast(uint4, a);
            const f16x8 al = __builtin_bit_cast(
                f16x8, make_uint4(grp < 2 ? au.x : 0u, grp == 0 ? au.y : (grp == 1 ? (au.y & 0xFFFFu) : 0u),
                                  grp == 0 ? au.z : 0u, grp == 0 ? au.w : 0u));
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, bh[nt], (f32x4){0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                d = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bl[nt], d, 0, 0, 0);
                mk[nt][2 * h] = mask_f16x2(d[0], d[1]);
                mk[nt][2 * h + 1] = mask_f16x2(d[2], d[3]);
                if (mask) {   // hidden 16 mt + 4 grp + j of query 16 nt + col: bits of half mt / 2
                    const uint32_t b4 = (d[0] > 0.f ? 1u : 0u) | (d[1] > 0.f ? 2u : 0u) | (d[2] > 0.f ? 4u : 0u) |
                                        (d[3] > 0.f ? 8u : 0u);
                    mbits[nt][ch] |= b4 << (16 * h + 4 * grp);
                }
            }
        }
        const f16x8 a2h = ((const f16x8*)(pk + kPkA2))[(2 * ch) * 64 + lane];
        const f16x8 a2l = ((const f16x8*)(pk + kPkA2))[(2 * ch + 1) * 64 + lane];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            const f16x8 b = __builtin_bit_cast(f16x8, make_uint4(mk[nt][0], mk[nt][1], mk[nt][2], mk[nt][3]));
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2h, b, acc[nt], 0, 0, 0);
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2l, b, acc[nt], 0, 0, 0);
        }
    }
    // ---- g back to the query's lane: lane (col, grp) holds rows 4grp..4grp+3 of query 16nt+col
    wave_lds_sync();   // every lane has read its B operands
    if (grp < 3) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) *(f32x4*)(xs + (16 * nt + col) * kXsStride + 4 * grp) = acc[nt];
    }
    wave_lds_sync();
    }
    if (mask) {
        // OR over the four lane groups (grp) holding a query's hidden rows; lane q = col + 16 grp
        // then holds query 16 nt + col's whole mask for every nt -- its own query at nt = grp
        uint32_t lo = 0u, hi = 0u;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            uint32_t a = mbits[nt][0], b = mbits[nt][1];
            a |= __shfl_xor(a, 16);
            a |= __shfl_xor(a, 32);
            b |= __shfl_xor(b, 16);
            b |= __shfl_xor(b, 32);
            lo = nt == grp ? a : lo;
            hi = nt == grp ? b : hi;
        }
        *mask = ((uint64_t)hi << 32) | lo;
    }
    const f32x4* r = (const f32x4*)(xs + lane * kXsStride);
    const f32x4 g0 = r[0], g1 = r[1], g2 = r[2];
    const f32x4* us = (const f32x4*)(pk + kPkScale);
    const f32x4 u0 = us[0], u1 = us[1], u2 = us[2];
    const float g[12] = {g0[0] * u0[0], g0[1] * u0[1], g0[2] * u0[2], g0[3] * u0[3],
                         g1[0] * u1[0], g1[1] * u1[1], g1[2] * u1[2], g1[3] * u1[3],
                         g2[0] * u2[0], g2[1] * u2[1], g2[2] * u2[2], g2[3] * u2[3]};
    wave_lds_sync();   // the next call's staging reuses xs
    float out = g[11] + *(const float*)(pk + kPkB2);
#pragma unroll
    for (int i = 0; i < kD; ++i) out = fmaf(x[i], g[i], out);
    if (GRAD) {
#pragma unroll
        for (int i = 0; i < NOUT; ++i) gx[i] = g[OFF + i] * m.sdf_scale;
    }
    return out * m.sdf_scale;
}

// The decoder's input gradient over the features from a given ReLU mask: gx[i] = s * sum_c
// 1[mask bit c] w2_c W1[c][i], i < 8 -- GEMM2 of mlp_sdf_mfma16 alone (16 MFMAs per wave, no
// GEMM1, no input staging).  The per-neighbour training backward takes each neighbour's mask from
// the forward's f32 decode (PIN_TRAIN_DX), so it neither re-gathers the neighbour's features nor
// re-evaluates its hidden layer.  All 64 lanes of the wave call this (lanes without a row pass 0).
__device__ __forceinline__ void mlp_grad8_from_mask(const MlpW& m, uint64_t mask, float (&gx)[kF]) {
    float* xs = m.xs;
    const unsigned char* pk = m.pk;
    const int lane = threadIdx.x & 63;
    const int col = lane & 15, grp = lane >> 4;
    wave_lds_sync();   // xs is the wave's scratch: every lane is past its earlier reads
    ((uint2*)xs)[lane] = make_uint2((uint32_t)mask, (uint32_t)(mask >> 32));
    wave_lds_sync();
    uint64_t qm[4];   // the masks of queries 16 nt + col
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const uint2 v = ((const uint2*)xs)[16 * nt + col];
        qm[nt] = ((uint64_t)v.y << 32) | v.x;
    }
    auto word = [](uint32_t b4, int p) -> uint32_t {   // two f16 halves: 1.0h where the bit is set
        return ((b4 >> (2 * p)) & 1u ? 0x3C00u : 0u) | ((b4 >> (2 * p + 1)) & 1u ? 0x3C000000u : 0u);
    };
    f32x4 acc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ch = 0; ch < 2; ++ch) {
        const f16x8 a2h = ((const f16x8*)(pk + kPkA2))[(2 * ch) * 64 + lane];
        const f16x8 a2l = ((const f16x8*)(pk + kPkA2))[(2 * ch + 1) * 64 + lane];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            // K-slot s of lane group grp <-> hidden 32 ch + (s < 4 ? 4 grp + s : 16 + 4 grp + s - 4)
            const uint32_t lo4 = (uint32_t)(qm[nt] >> (32 * ch + 4 * grp)) & 15u;
            const uint32_t hi4 = (uint32_t)(qm[nt] >> (32 * ch + 16 + 4 * grp)) & 15u;
            const f16x8 b = __builtin_bit_cast(f16x8, make_uint4(word(lo4, 0), word(lo4, 1), word(hi4, 0), word(hi4, 1)));
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2h, b, acc[nt], 0, 0, 0);
            acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a2l, b, acc[nt], 0, 0, 0);
        }
    }
    // rows 4 grp .. 4 grp + 3 of query 16 nt + col back to the query's lane (rows 0..7 are used)
    wave_lds_sync();   // every lane has read the masks
    if (grp < 2) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) *(f32x4*)(xs + (16 * nt + col) * kXsStride + 4 * grp) = acc[nt];
    }
    wave_lds_sync();
    const f32x4* r = (const f32x4*)(xs + lane * kXsStride);
    const f32x4 g0 = r[0], g1 = r[1];
    const f32x4* us = (const f32x4*)(pk + kPkScale);
    const f32x4 u0 = us[0], u1 = us[1];
    gx[0] = g0[0] * u0[0] * m.sdf_scale; gx[1] = g0[1] * u0[1] * m.sdf_scale;
    gx[2] = g0[2] * u0[2] * m.sdf_scale; gx[3] = g0[3] * u0[3] * m.sdf_scale;
    gx[4] = g1[0] * u1[0] * m.sdf_scale; gx[5] = g1[1] * u1[1] * m.sdf_scale;
    gx[6] = g1[2] * u1[2] * m.sdf_scale; gx[7] = g1[3] * u1[3] * m.sdf_scale;
    wave_lds_sync();   // the next call reuses xs
}

// Block setup of the decoder (all threads; ends with a barrier): the f32 weights, or (MF) the
// pin_mlp_pack image, with each wave's scan list as the scratch of mlp_sdf_mfma16.
static_assert(kXsWave <= kListSeg * 64, "decoder scratch must fit the wave's scan list");

template <bool MF>
__device__ __forceinline__ MlpW stage_decoder(const PinMlp& m, float* s_mlp, uint4* s_pk) {
    if constexpr (MF) {
        const uint4* src = (const uint4*)m.packed;
        for (int e = threadIdx.x; e < kPkBytes / 16; e += blockDim.x) s_pk[e] = src[e];
        __syncthreads();
        return MlpW{nullptr, m.sdf_scale, (float*)wave_list(), (const unsigned char*)s_pk};
    } else {
        return stage_mlp(m, s_mlp);
    }
}

}  // namespace pin
