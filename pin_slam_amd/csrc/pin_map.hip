// pin_map.hip -- map maintenance of NeuralPoints on the device:
// voxel down-sampling, hash insert with the reference's collision / staleness rules,
// local-map selection, pruning, pose adjustment and re-hashing
// (model/neural_points.py:205-428, utils/tools.py:326-477).
//
// Everything here is integer / byte work bounded by HBM and launch latency: per-point
// kernels with coalesced loads, rocPRIM for the one sort (voxel keys) and the stream
// compactions (inclusive scans), no host round trip inside a call.
//
// Exactness rules followed (they decide which point survives and which id it gets):
//   * voxel coordinates are floor(p / res) with IEEE f32 division, as on the CPU path;
//   * float -> int64 conversions follow x86 cvttss2si: truncation, NaN / out of range ->
//     INT64_MIN (what torch's CPU .long() produces for the quantised 0/0 levels);
//   * the packed "index + level * 10^digits" arithmetic wraps like int64 tensors do;
//   * a slot written by several points of one call keeps the last one (CPU index_put order):
//     claimed with atomicMin on a marker INT_MIN + (n - 1 - i), then written by its winner.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstring>
#include <stdint.h>

#include <algorithm>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "pin_device.h"

using namespace pin;

namespace {

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline unsigned blocks_for(int64_t n, int per = kBlock) { return (unsigned)((n + per - 1) / per); }
inline int status(hipError_t e) { return (e == hipSuccess && hipGetLastError() == hipSuccess) ? PIN_OK : PIN_ERR_HIP; }

// ----------------------------------------------------------------------------- numerics
// torch CPU float -> int64 (.long()): truncation; NaN, +-inf and |x| >= 2^63 give INT64_MIN
__device__ __forceinline__ int64_t to_long(float x) {
    if (!(x >= -0x1p63f && x < 0x1p63f)) return LLONG_MIN;
    return (int64_t)x;
}

__device__ __forceinline__ int64_t wrap_add_mul(int64_t a, int64_t b, int64_t c) {  // a + b * c mod 2^64
    return (int64_t)((uint64_t)a + (uint64_t)b * (uint64_t)c);
}

// order-preserving map of floats onto signed ints, for an atomicMax over floats of any sign
__device__ __forceinline__ int float_order(float f) {
    const int b = __float_as_int(f);
    return b >= 0 ? b : b ^ 0x7fffffff;
}
__device__ __forceinline__ float order_float(int o) { return __int_as_float(o >= 0 ? o : o ^ 0x7fffffff); }

// utils/tools.py:423-427: distance of a point to the centre of its voxel, reference op order
__device__ __forceinline__ float centre_dist(float px, float py, float pz, float vs) {
    const float cx = (floorf(px / vs) + 0.5f) * vs, cy = (floorf(py / vs) + 0.5f) * vs,
                cz = (floorf(pz / vs) + 0.5f) * vs;
    const float dx = px - cx, dy = py - cy, dz = pz - cz;
    return sqrtf((dx * dx + dy * dy) + dz * dz);
}

// ----------------------------------------------------------------------------- workspace
constexpr int64_t kAlign = 256;
inline int64_t align_up(int64_t b) { return (b + kAlign - 1) / kAlign * kAlign; }

// rocPRIM temporary-storage sizes (0 when the query fails, e.g. without a device)
size_t sort_temp_bytes(int64_t n) {
    size_t bytes = 0;
    if (rocprim::radix_sort_pairs(nullptr, bytes, (uint64_t*)nullptr, (uint64_t*)nullptr, (int64_t*)nullptr,
                                  (int64_t*)nullptr, (size_t)std::max<int64_t>(n, 1), 0, 64,
                                  (hipStream_t)0) != hipSuccess)
        return 0;
    return bytes;
}

size_t scan_temp_bytes(int64_t n) {
    size_t bytes = 0;
    if (rocprim::inclusive_scan(nullptr, bytes, (const int32_t*)nullptr, (int64_t*)nullptr,
                                (size_t)std::max<int64_t>(n, 1), rocprim::plus<int64_t>(),
                                (hipStream_t)0) != hipSuccess)
        return 0;
    return bytes;
}

// The carve-up shared by every call: a bump allocator over the caller's workspace
struct Carve {
    char* p;
    template <class T>
    T* take(int64_t count) {
        T* r = (T*)p;
        p += align_up((int64_t)sizeof(T) * std::max<int64_t>(count, 1));
        return r;
    }
};

struct VdsStats {          // device-side reduction results of the down-sampler
    long long lo[3];       // min voxel coordinate per axis
    long long hi[3];       // max voxel coordinate per axis
    int vmax;              // float_order(max level source: distance or value)
    int pad;
};

hipError_t incl_scan(void* tmp, size_t bytes, const int32_t* flags, int64_t* incl, int64_t n, hipStream_t s) {
    return rocprim::inclusive_scan(tmp, bytes, flags, incl, (size_t)n, rocprim::plus<int64_t>(), s);
}

// ----------------------------------------------------------------------------- down-sample
__global__ void k_vds_init(VdsStats* st) {
    if (threadIdx.x < 3) {
        st->lo[threadIdx.x] = LLONG_MAX;
        st->hi[threadIdx.x] = LLONG_MIN;
    }
    if (threadIdx.x == 0) st->vmax = INT_MIN;
}

__global__ void __launch_bounds__(kBlock)
k_vds_stats(const float* __restrict__ pts, int64_t n, float vs, const float* __restrict__ value,
            VdsStats* __restrict__ st) {
    long long lo[3] = {LLONG_MAX, LLONG_MAX, LLONG_MAX}, hi[3] = {LLONG_MIN, LLONG_MIN, LLONG_MIN};
    int vm = INT_MIN;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        const float p[3] = {pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]};
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const long long c = (long long)floorf(p[a] / vs);
            lo[a] = c < lo[a] ? c : lo[a];
            hi[a] = c > hi[a] ? c : hi[a];
        }
        const float v = value ? value[i] : centre_dist(p[0], p[1], p[2], vs);
        vm = max(vm, float_order(v));
    }
    __shared__ long long red[kBlock / 64][6];
    __shared__ int redv[kBlock / 64];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        for (int off = 32; off > 0; off >>= 1) {
            const long long l = __shfl_xor(lo[a], off), h = __shfl_xor(hi[a], off);
            lo[a] = l < lo[a] ? l : lo[a];
            hi[a] = h > hi[a] ? h : hi[a];
        }
    }
    for (int off = 32; off > 0; off >>= 1) vm = max(vm, __shfl_xor(vm, off));
    if ((threadIdx.x & 63) == 0) {
        const int w = threadIdx.x >> 6;
        for (int a = 0; a < 3; ++a) {
            red[w][a] = lo[a];
            red[w][3 + a] = hi[a];
        }
        redv[w] = vm;
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        long long v = red[0][threadIdx.x];
        for (int w = 1; w < kBlock / 64; ++w) {
            const long long t = red[w][threadIdx.x];
            v = threadIdx.x < 3 ? (t < v ? t : v) : (t > v ? t : v);
        }
        if (threadIdx.x < 3) atomicMin(&st->lo[threadIdx.x], v);
        else atomicMax(&st->hi[threadIdx.x - 3], v);
    } else if (threadIdx.x == 6) {
        int v = redv[0];
        for (int w = 1; w < kBlock / 64; ++w) v = max(v, redv[w]);
        atomicMax(&st->vmax, v);
    }
}

// key = c0 + c1 v + c2 v^2 with c = voxel - min voxel and v = grid.max() (tools.py:428-431);
// packed = i + long(level) * scale (tools.py:434-437)
__global__ void __launch_bounds__(kBlock)
k_vds_keys(const float* __restrict__ pts, int64_t n, float vs, const float* __restrict__ value,
           const VdsStats* __restrict__ st, int64_t scale, uint64_t* __restrict__ keys, int64_t* __restrict__ packed) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float px = pts[3 * i], py = pts[3 * i + 1], pz = pts[3 * i + 2];
    const long long c0 = (long long)floorf(px / vs) - st->lo[0];
    const long long c1 = (long long)floorf(py / vs) - st->lo[1];
    const long long c2 = (long long)floorf(pz / vs) - st->lo[2];
    long long v = st->hi[0] - st->lo[0];
    v = max(v, st->hi[1] - st->lo[1]);
    v = max(v, st->hi[2] - st->lo[2]);
    keys[i] = (uint64_t)(c0 + c1 * v + c2 * v * v);
    const float vmax = order_float(st->vmax);
    const float src = value ? value[i] : centre_dist(px, py, pz, vs);
    const float level = src / vmax * 999.f;
    packed[i] = wrap_add_mul(i, to_long(level), scale);
}

__global__ void __launch_bounds__(kBlock)
k_run_flags(const uint64_t* __restrict__ keys, int64_t n, int32_t* __restrict__ flags) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    flags[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1 : 0;
}

// one thread per run of equal keys: amin of the packed values, then the Python-style
// remainder by scale (torch's % on int64) recovers the index
__global__ void __launch_bounds__(kBlock)
k_vds_runs(const uint64_t* __restrict__ keys, const int64_t* __restrict__ packed, const int32_t* __restrict__ flags,
           const int64_t* __restrict__ incl, int64_t n, int64_t scale, int64_t* __restrict__ out,
           int64_t* __restrict__ count) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    if (i == n - 1) *count = incl[n - 1];
    if (!flags[i]) return;
    const uint64_t k = keys[i];
    int64_t m = packed[i];
    for (int64_t j = i + 1; j < n && keys[j] == k; ++j) m = min(m, packed[j]);
    int64_t r = m % scale;
    if (r < 0) r += scale;
    out[incl[i] - 1] = r;
}

// ----------------------------------------------------------------------------- hash writes
// last-writer claim: the smallest marker = the largest i
__device__ __forceinline__ int claim_marker(int64_t i, int64_t n) { return INT_MIN + (int)(n - 1 - i); }

__device__ __forceinline__ float3 load_row3(const float* __restrict__ pts, const int64_t* __restrict__ rows,
                                            int64_t i) {
    const int64_t r = rows ? rows[i] : i;
    return make_float3(pts[3 * r], pts[3 * r + 1], pts[3 * r + 2]);
}

// neural_points.py:214-231: slot, current entry and the insert decision of each sample
__global__ void __launch_bounds__(kBlock)
k_insert_probe(const float* __restrict__ pts, const int64_t* __restrict__ rows, int64_t n, float res,
               const int32_t* __restrict__ table, int64_t B, const float* __restrict__ pos,
               const int64_t* __restrict__ ts_update, int64_t count, const float* __restrict__ td, int64_t cur_ts,
               float dist2_thre, float travel_thre, int32_t* __restrict__ slot_out, int32_t* __restrict__ hidx_out,
               int32_t* __restrict__ flags) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float3 p = load_row3(pts, rows, i);
    const uint32_t s = base_slot(p.x, p.y, p.z, res, B);
    const int h = table[s];
    bool fresh = true;
    if (count > 0 && h >= 0) {
        const float d2 = dist2(pos[3 * (int64_t)h], pos[3 * (int64_t)h + 1], pos[3 * (int64_t)h + 2], p.x, p.y, p.z);
        const float dtd = td[cur_ts] - td[ts_update[h]];
        fresh = d2 > dist2_thre || dtd > travel_thre;
    }
    slot_out[i] = (int32_t)s;
    hidx_out[i] = h;
    flags[i] = fresh ? 1 : 0;
}

__global__ void __launch_bounds__(kBlock)
k_claim(const int32_t* __restrict__ slots, int64_t n, int32_t* __restrict__ table) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    atomicMin(table + slots[i], claim_marker(i, n));
}

// the winner of each claimed slot writes its entry; new points are listed in id order
__global__ void __launch_bounds__(kBlock)
k_insert_write(const int32_t* __restrict__ slots, const int32_t* __restrict__ hidx, const int32_t* __restrict__ flags,
               const int64_t* __restrict__ incl, const int64_t* __restrict__ rows, int64_t n, int64_t count,
               int32_t* __restrict__ table, int64_t* __restrict__ new_rows, int64_t* __restrict__ n_new) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    if (i == n - 1) *n_new = incl[n - 1];
    const bool fresh = flags[i] != 0;
    const int64_t rank = incl[i] - 1;
    const int32_t cur = fresh ? (int32_t)(count + rank) : hidx[i];
    if (table[slots[i]] == claim_marker(i, n)) table[slots[i]] = cur;
    if (fresh) new_rows[rank] = rows ? rows[i] : i;
}

__global__ void __launch_bounds__(kBlock)
k_assign_slots(const float* __restrict__ pts, const int64_t* __restrict__ rows, int64_t n, float res, int64_t B,
               int32_t* __restrict__ slots, int32_t* __restrict__ table) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float3 p = load_row3(pts, rows, i);
    const uint32_t s = base_slot(p.x, p.y, p.z, res, B);
    slots[i] = (int32_t)s;
    atomicMin(table + s, claim_marker(i, n));
}

__global__ void __launch_bounds__(kBlock)
k_assign_write(const int32_t* __restrict__ slots, const int64_t* __restrict__ rows, int64_t n,
               int32_t* __restrict__ table) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    if (table[slots[i]] == claim_marker(i, n)) table[slots[i]] = (int32_t)(rows ? rows[i] : i);
}

// ----------------------------------------------------------------------------- local map / prune
// ((create + update) / 2).long(): int64 sum, true division to the default float dtype, truncation
__device__ __forceinline__ int64_t ts_used(const int64_t* __restrict__ tc, const int64_t* __restrict__ tu,
                                           int64_t i, bool mid) {
    return mid ? to_long((float)(tc[i] + tu[i]) / 2.f) : tc[i];
}

template <class S>
__global__ void __launch_bounds__(kBlock)
k_local_flags(const float* __restrict__ pos, const int64_t* __restrict__ tc, const int64_t* __restrict__ tu,
              int64_t count, const float* __restrict__ td, const S* __restrict__ sensor, int64_t cur_ts, S radius2,
              float travel_thre, int mid, int use_td, int64_t diff_ts, int32_t* __restrict__ flags) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= count) return;
    const S dx = (S)pos[3 * i] - sensor[0], dy = (S)pos[3 * i + 1] - sensor[1], dz = (S)pos[3 * i + 2] - sensor[2];
    const S d2 = (dx * dx + dy * dy) + dz * dz;
    const int64_t t = ts_used(tc, tu, i, mid);
    bool near_t;
    if (use_td) {
        near_t = fabsf(td[cur_ts] - td[t]) < travel_thre;
    } else {
        const int64_t dt = cur_ts - t;
        near_t = (dt < 0 ? -dt : dt) < diff_ts;
    }
    flags[i] = (d2 < radius2 && near_t) ? 1 : 0;
}

__global__ void __launch_bounds__(kBlock)
k_local_write(const int32_t* __restrict__ flags, const int64_t* __restrict__ incl, int64_t count, int64_t fill,
              uint8_t* __restrict__ mask, int64_t* __restrict__ g2l, int64_t* __restrict__ rows,
              int64_t* __restrict__ n_out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i > count) return;
    if (i == count) {  // the padding entry
        if (mask) mask[count] = 1;
        if (g2l) g2l[count] = -1;
        *n_out = count > 0 ? incl[count - 1] : 0;
        return;
    }
    const bool in = flags[i] != 0;
    const int64_t rank = incl[i] - 1;
    if (mask) mask[i] = in ? 1 : 0;
    if (g2l) g2l[i] = in ? rank : fill;
    if (in) rows[rank] = i;
}

__global__ void __launch_bounds__(kBlock)
k_keep_flags(const int64_t* __restrict__ tu, const float* __restrict__ cert, int64_t count,
             const float* __restrict__ td, int64_t cur_ts, float travel_thre, float cert_thre,
             int32_t* __restrict__ flags) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= count) return;
    const bool inactive = fabsf(td[cur_ts] - td[tu[i]]) > travel_thre;
    flags[i] = (inactive && cert[i] < cert_thre) ? 0 : 1;
}

// ----------------------------------------------------------------------------- pool window filter
// utils/mapper.py:226-233: torch.sum((coord - origin) ** 2, dim=-1) < window_radius ** 2 with
// torch's type promotion: an f64 pose makes the difference, squares, sum and bound f64; an f32
// pose keeps them f32 (the bound rounded to f32); the three-term sum in the reference's order
template <typename T>
__global__ void __launch_bounds__(kBlock)
k_window_flags(const float* __restrict__ coord, int64_t n, const T* __restrict__ center, T r2,
               int32_t* __restrict__ flags) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const T dx = (T)coord[3 * i] - center[0], dy = (T)coord[3 * i + 1] - center[1], dz = (T)coord[3 * i + 2] - center[2];
    const T d2 = (dx * dx + dy * dy) + dz * dz;
    flags[i] = d2 < r2 ? 1 : 0;
}

// kept rows in order, and counts = {kept rows, kept rows at index >= tail_start}
__global__ void __launch_bounds__(kBlock)
k_window_write(const int32_t* __restrict__ flags, const int64_t* __restrict__ incl, int64_t n, int64_t tail_start,
               int64_t* __restrict__ keep, int64_t* __restrict__ counts) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i > n) return;
    if (i == n) {
        const int64_t total = n > 0 ? incl[n - 1] : 0;
        const int64_t t = tail_start < 0 ? 0 : tail_start > n ? n : tail_start;
        counts[0] = total;
        counts[1] = total - (t > 0 ? incl[t - 1] : 0);
        return;
    }
    if (flags[i]) keep[incl[i] - 1] = i;
}

// ----------------------------------------------------------------------------- gather / scatter
// One thread per row: every array of the row moves with 16/8/4-byte loads and stores.  The
// local / kept row lists are ascending, so neighbouring lanes touch neighbouring rows.
template <bool SCATTER>
__global__ void __launch_bounds__(kBlock)
k_move_rows(const int64_t* __restrict__ rows, int64_t n_rows, PinMapArrays src, PinMapArrays dst, uint32_t sel,
            int F) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n_rows) return;
    const int64_t r = rows[i];
    if (r < 0) {   // no source row: a gather writes zeros, a scatter skips
        if (SCATTER) return;
        const int64_t d = i;
        if (sel & 1) dst.positions[3 * d] = dst.positions[3 * d + 1] = dst.positions[3 * d + 2] = 0.f;
        if (sel & 2) ((float4*)dst.orientations)[d] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (sel & 4) dst.ts_create[d] = 0;
        if (sel & 8) dst.ts_update[d] = 0;
        if (sel & 16) dst.certainties[d] = 0.f;
        if (sel & 32)
            for (int k = 0; k < F; ++k) dst.features[(int64_t)F * d + k] = 0.f;
        return;
    }
    const int64_t s = SCATTER ? i : r, d = SCATTER ? r : i;
    if (sel & 1) {
        const float* a = src.positions + 3 * s;
        float* b = dst.positions + 3 * d;
        const float x = a[0], y = a[1], z = a[2];
        b[0] = x;
        b[1] = y;
        b[2] = z;
    }
    if (sel & 2) ((float4*)dst.orientations)[d] = ((const float4*)src.orientations)[s];
    if (sel & 4) dst.ts_create[d] = src.ts_create[s];
    if (sel & 8) dst.ts_update[d] = src.ts_update[s];
    if (sel & 16) dst.certainties[d] = src.certainties[s];
    if (sel & 32) {
        if (F == 8) {
            const float4* a = (const float4*)(src.features + 8 * s);
            float4* b = (float4*)(dst.features + 8 * d);
            const float4 u = a[0], v = a[1];
            b[0] = u;
            b[1] = v;
        } else {
            for (int k = 0; k < F; ++k) dst.features[(int64_t)F * d + k] = src.features[(int64_t)F * s + k];
        }
    }
}

__global__ void k_copy_words(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, int words) {
    if ((int)threadIdx.x < words) dst[threadIdx.x] = src[threadIdx.x];
}

int move_rows(const PinMapArrays* src, const PinMapArrays* dst, const int64_t* rows, int64_t n_rows, int pad_row,
              bool scatter, hipStream_t s) {
    if (!src || !dst || n_rows < 0 || (n_rows > 0 && !rows)) return PIN_ERR_ARG;
    const PinMapArrays* sel = scatter ? src : dst;  // which side's non-NULL arrays choose what moves
    const void* a[6] = {src->positions, src->orientations, src->ts_create, src->ts_update, src->certainties,
                        src->features};
    const void* b[6] = {dst->positions, dst->orientations, dst->ts_create, dst->ts_update, dst->certainties,
                        dst->features};
    const void* c[6] = {sel->positions, sel->orientations, sel->ts_create, sel->ts_update, sel->certainties,
                        sel->features};
    uint32_t mask = 0;
    for (int k = 0; k < 6; ++k) {
        if (!c[k]) continue;
        if (!a[k] || !b[k]) return PIN_ERR_ARG;
        mask |= 1u << k;
    }
    const int F = sel->feature_dim > 0 ? sel->feature_dim : kF;
    if (mask && n_rows > 0)
        hipLaunchKernelGGL(scatter ? k_move_rows<true> : k_move_rows<false>, dim3(blocks_for(n_rows)), dim3(kBlock),
                           0, s, rows, n_rows, *src, *dst, mask, F);
    if (pad_row && (mask & 32)) {
        const int64_t srow = scatter ? n_rows : src->count, drow = scatter ? dst->count : n_rows;
        hipLaunchKernelGGL(k_copy_words, dim3(1), dim3(64), 0, s, (const uint32_t*)(src->features + srow * F),
                           (uint32_t*)(dst->features + drow * F), F);
    }
    return status(hipSuccess);
}

// ----------------------------------------------------------------------------- multi-array gather
struct RowArrays {
    const unsigned char* src[PIN_ROW_ARRAYS_MAX];
    unsigned char* dst[PIN_ROW_ARRAYS_MAX];
    int64_t units[PIN_ROW_ARRAYS_MAX];   // accesses per row
    int32_t shift[PIN_ROW_ARRAYS_MAX];   // log2 of the access width: 4 (16 B), 3, 2 or 0
    int32_t n;
};

template <typename T>
__device__ __forceinline__ void copy_units(const unsigned char* s, unsigned char* d, int64_t units) {
    const T* a = (const T*)s;
    T* b = (T*)d;
    for (int64_t u = 0; u < units; ++u) b[u] = a[u];
}

// one thread per output row, every array: the kept-row list is ascending, so neighbouring lanes
// read neighbouring source rows
__global__ void __launch_bounds__(kBlock)
k_gather_rows(RowArrays A, const int64_t* __restrict__ rows, int64_t n_rows) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n_rows) return;
    const int64_t r = rows[i];
    for (int a = 0; a < A.n; ++a) {
        const int64_t units = A.units[a];
        const int sh = A.shift[a];
        const int64_t bytes = units << sh;
        const unsigned char* s = A.src[a] + r * bytes;
        unsigned char* d = A.dst[a] + i * bytes;
        switch (sh) {
            case 4: copy_units<uint4>(s, d, units); break;
            case 3: copy_units<uint2>(s, d, units); break;
            case 2: copy_units<uint32_t>(s, d, units); break;
            default: copy_units<unsigned char>(s, d, units); break;
        }
    }
}

// ----------------------------------------------------------------------------- pose adjustment
// utils/tools.py:326-334 rotmat_to_quat, :356-369 quat_multiply, :401-407 transform_batch_torch
__global__ void __launch_bounds__(kBlock)
k_map_adjust(float* __restrict__ pos, float* __restrict__ quat, const int64_t* __restrict__ tc,
             const int64_t* __restrict__ tu, int64_t count, const float* __restrict__ T, int mid) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= count) return;
    const float* M = T + 16 * ts_used(tc, tu, i, mid);
    const float x = pos[3 * i], y = pos[3 * i + 1], z = pos[3 * i + 2];
    pos[3 * i] = ((M[0] * x + M[1] * y) + M[2] * z) + M[3];
    pos[3 * i + 1] = ((M[4] * x + M[5] * y) + M[6] * z) + M[7];
    pos[3 * i + 2] = ((M[8] * x + M[9] * y) + M[10] * z) + M[11];
    if (!quat) return;
    const float w1 = sqrtf(((1.0f + M[0]) + M[5]) + M[10]) / 2.0f;
    const float x1 = (M[9] - M[6]) / (4.0f * w1);
    const float y1 = (M[2] - M[8]) / (4.0f * w1);
    const float z1 = (M[4] - M[1]) / (4.0f * w1);
    const float w2 = quat[4 * i], x2 = quat[4 * i + 1], y2 = quat[4 * i + 2], z2 = quat[4 * i + 3];
    quat[4 * i] = ((w1 * w2 - x1 * x2) - y1 * y2) - z1 * z2;
    quat[4 * i + 1] = ((w1 * x2 + x1 * w2) + y1 * z2) - z1 * y2;
    quat[4 * i + 2] = ((w1 * y2 - x1 * z2) + y1 * w2) + z1 * x2;
    quat[4 * i + 3] = ((w1 * z2 + x1 * y2) - y1 * x2) + z1 * w2;
}

}  // namespace

extern "C" {

int64_t pin_map_workspace_bytes(int64_t n) {
    n = std::max<int64_t>(n, 1);
    const int64_t temp = (int64_t)std::max(sort_temp_bytes(n), scan_temp_bytes(n + 1));
    if (temp == 0) return PIN_ERR_HIP;
    // keys x2, packed x2 (8 B), flags, slots, hidx (4 B), incl (8 B), stats, rocPRIM temp
    return 4 * align_up(8 * n) + 3 * align_up(4 * n) + align_up(8 * (n + 1)) + align_up(sizeof(VdsStats)) +
           align_up(temp) + kAlign;
}

int pin_voxel_down_sample(const float* points, int64_t n, float voxel_size, const float* value, int64_t* out_idx,
                          int64_t* count, void* workspace, void* stream) {
    if (!points || n <= 0 || !out_idx || !count || !workspace || !(voxel_size > 0.f)) return PIN_ERR_ARG;
    auto s = as_stream(stream);
    Carve c{(char*)workspace};
    uint64_t* keys_a = c.take<uint64_t>(n);
    uint64_t* keys_b = c.take<uint64_t>(n);
    int64_t* pk_a = c.take<int64_t>(n);
    int64_t* pk_b = c.take<int64_t>(n);
    int32_t* flags = c.take<int32_t>(n);
    c.take<int32_t>(n);
    c.take<int32_t>(n);
    int64_t* incl = c.take<int64_t>(n + 1);
    VdsStats* st = c.take<VdsStats>(1);
    const size_t temp_bytes = std::max(sort_temp_bytes(n), scan_temp_bytes(n + 1));
    void* temp = c.take<char>((int64_t)temp_bytes);
    // offset = 10 ** len(str(n - 1))
    int64_t scale = 10;
    for (int64_t m = n - 1; m >= 10; m /= 10) scale *= 10;
    hipLaunchKernelGGL(k_vds_init, dim3(1), dim3(64), 0, s, st);
    hipLaunchKernelGGL(k_vds_stats, dim3((unsigned)std::min<int64_t>(blocks_for(n), 128)), dim3(kBlock), 0, s,
                       points, n, voxel_size, value, st);
    hipLaunchKernelGGL(k_vds_keys, dim3(blocks_for(n)), dim3(kBlock), 0, s, points, n, voxel_size, value, st, scale,
                       keys_a, pk_a);
    size_t tb = temp_bytes;
    hipError_t e = rocprim::radix_sort_pairs(temp, tb, keys_a, keys_b, pk_a, pk_b, (size_t)n, 0, 64, s);
    if (e != hipSuccess) return PIN_ERR_HIP;
    hipLaunchKernelGGL(k_run_flags, dim3(blocks_for(n)), dim3(kBlock), 0, s, keys_b, n, flags);
    tb = temp_bytes;
    if (incl_scan(temp, tb, flags, incl, n, s) != hipSuccess) return PIN_ERR_HIP;
    hipLaunchKernelGGL(k_vds_runs, dim3(blocks_for(n)), dim3(kBlock), 0, s, keys_b, pk_b, flags, incl, n, scale,
                       out_idx, count);
    return status(hipSuccess);
}

int pin_map_insert(const float* points, const int64_t* sample_idx, int64_t n, float resolution, int32_t* table,
                   int64_t buffer_size, const float* positions, const int64_t* ts_update, int64_t count,
                   const float* travel_dist, int64_t cur_ts, float dist2_thre, float travel_thre, int64_t* new_rows,
                   int64_t* n_new, void* workspace, void* stream) {
    if (!points || n < 0 || !table || buffer_size <= 0 || buffer_size >= (1ll << 31) || !new_rows || !n_new ||
        !workspace || count < 0 || count + n >= (1ll << 31) || !(resolution > 0.f))
        return PIN_ERR_ARG;
    if (count > 0 && (!positions || !ts_update || !travel_dist)) return PIN_ERR_ARG;
    auto s = as_stream(stream);
    if (n == 0) return status(hipMemsetAsync(n_new, 0, sizeof(int64_t), s));
    Carve c{(char*)workspace};
    c.take<uint64_t>(n);
    c.take<uint64_t>(n);
    c.take<int64_t>(n);
    c.take<int64_t>(n);
    int32_t* flags = c.take<int32_t>(n);
    int32_t* slots = c.take<int32_t>(n);
    int32_t* hidx = c.take<int32_t>(n);
    int64_t* incl = c.take<int64_t>(n + 1);
    c.take<VdsStats>(1);
    const size_t temp_bytes = std::max(sort_temp_bytes(n), scan_temp_bytes(n + 1));
    void* temp = c.take<char>((int64_t)temp_bytes);
    hipLaunchKernelGGL(k_insert_probe, dim3(blocks_for(n)), dim3(kBlock), 0, s, points, sample_idx, n, resolution,
                       table, buffer_size, positions, ts_update, count, travel_dist, cur_ts, dist2_thre, travel_thre,
                       slots, hidx, flags);
    size_t tb = temp_bytes;
    if (incl_scan(temp, tb, flags, incl, n, s) != hipSuccess) return PIN_ERR_HIP;
    hipLaunchKernelGGL(k_claim, dim3(blocks_for(n)), dim3(kBlock), 0, s, slots, n, table);
    hipLaunchKernelGGL(k_insert_write, dim3(blocks_for(n)), dim3(kBlock), 0, s, slots, hidx, flags, incl, sample_idx,
                       n, count, table, new_rows, n_new);
    return status(hipSuccess);
}

int pin_hash_assign(const float* points, const int64_t* rows, int64_t n, float resolution, int32_t* table,
                    int64_t buffer_size, void* workspace, void* stream) {
    if (!points || n < 0 || n >= (1ll << 31) || !table || buffer_size <= 0 || buffer_size >= (1ll << 31) ||
        !workspace || !(resolution > 0.f))
        return PIN_ERR_ARG;
    if (n == 0) return PIN_OK;
    auto s = as_stream(stream);
    Carve c{(char*)workspace};
    c.take<uint64_t>(n);
    c.take<uint64_t>(n);
    c.take<int64_t>(n);
    c.take<int64_t>(n);
    c.take<int32_t>(n);
    int32_t* slots = c.take<int32_t>(n);
    hipLaunchKernelGGL(k_assign_slots, dim3(blocks_for(n)), dim3(kBlock), 0, s, points, rows, n, resolution,
                       buffer_size, slots, table);
    hipLaunchKernelGGL(k_assign_write, dim3(blocks_for(n)), dim3(kBlock), 0, s, slots, rows, n, table);
    return status(hipSuccess);
}

int pin_local_map(const PinMapArrays* map, const float* travel_dist, const void* sensor_position, int32_t sensor_f64,
                  int64_t cur_ts, double radius2, float travel_thre, int32_t use_mid_ts, int32_t use_travel_dist,
                  int64_t diff_ts_local, int64_t g2l_fill, uint8_t* local_mask, int64_t* global2local,
                  int64_t* local_rows, int64_t* local_count, void* workspace, void* stream) {
    if (!map || map->count < 0 || !sensor_position || !local_rows || !local_count || !workspace) return PIN_ERR_ARG;
    const int64_t M = map->count;
    if (M > 0 && (!map->positions || !map->ts_create || (use_mid_ts && !map->ts_update) ||
                  (use_travel_dist && !travel_dist)))
        return PIN_ERR_ARG;
    auto s = as_stream(stream);
    Carve c{(char*)workspace};
    c.take<uint64_t>(M);
    c.take<uint64_t>(M);
    c.take<int64_t>(M);
    c.take<int64_t>(M);
    int32_t* flags = c.take<int32_t>(M);
    c.take<int32_t>(M);
    c.take<int32_t>(M);
    int64_t* incl = c.take<int64_t>(M + 1);
    c.take<VdsStats>(1);
    const size_t temp_bytes = std::max(sort_temp_bytes(M), scan_temp_bytes(M + 1));
    void* temp = c.take<char>((int64_t)temp_bytes);
    if (M > 0) {
        if (sensor_f64)
            hipLaunchKernelGGL(k_local_flags<double>, dim3(blocks_for(M)), dim3(kBlock), 0, s, map->positions,
                               map->ts_create, map->ts_update, M, travel_dist, (const double*)sensor_position, cur_ts,
                               radius2, travel_thre, use_mid_ts, use_travel_dist, diff_ts_local, flags);
        else
            hipLaunchKernelGGL(k_local_flags<float>, dim3(blocks_for(M)), dim3(kBlock), 0, s, map->positions,
                               map->ts_create, map->ts_update, M, travel_dist, (const float*)sensor_position, cur_ts,
                               (float)radius2, travel_thre, use_mid_ts, use_travel_dist, diff_ts_local, flags);
        size_t tb = temp_bytes;
        if (incl_scan(temp, tb, flags, incl, M, s) != hipSuccess) return PIN_ERR_HIP;
    }
    hipLaunchKernelGGL(k_local_write, dim3(blocks_for(M + 1)), dim3(kBlock), 0, s, flags, incl, M, g2l_fill,
                       local_mask, global2local, local_rows, local_count);
    return status(hipSuccess);
}

int pin_prune_rows(const PinMapArrays* map, const float* travel_dist, int64_t cur_ts, float travel_thre,
                   float certainty_thre, int64_t* keep_rows, int64_t* keep_count, void* workspace, void* stream) {
    if (!map || map->count < 0 || !keep_rows || !keep_count || !workspace) return PIN_ERR_ARG;
    const int64_t M = map->count;
    if (M > 0 && (!map->ts_update || !map->certainties || !travel_dist)) return PIN_ERR_ARG;
    auto s = as_stream(stream);
    Carve c{(char*)workspace};
    c.take<uint64_t>(M);
    c.take<uint64_t>(M);
    c.take<int64_t>(M);
    c.take<int64_t>(M);
    int32_t* flags = c.take<int32_t>(M);
    c.take<int32_t>(M);
    c.take<int32_t>(M);
    int64_t* incl = c.take<int64_t>(M + 1);
    c.take<VdsStats>(1);
    const size_t temp_bytes = std::max(sort_temp_bytes(M), scan_temp_bytes(M + 1));
    void* temp = c.take<char>((int64_t)temp_bytes);
    if (M > 0) {
        hipLaunchKernelGGL(k_keep_flags, dim3(blocks_for(M)), dim3(kBlock), 0, s, map->ts_update, map->certainties, M,
                           travel_dist, cur_ts, travel_thre, certainty_thre, flags);
        size_t tb = temp_bytes;
        if (incl_scan(temp, tb, flags, incl, M, s) != hipSuccess) return PIN_ERR_HIP;
    }
    hipLaunchKernelGGL(k_local_write, dim3(blocks_for(M + 1)), dim3(kBlock), 0, s, flags, incl, M, (int64_t)0,
                       (uint8_t*)nullptr, (int64_t*)nullptr, keep_rows, keep_count);
    return status(hipSuccess);
}

int64_t pin_pool_window_workspace_bytes(int64_t n) {
    n = std::max<int64_t>(n, 1);
    return align_up(4 * n) + align_up(8 * (n + 1)) + align_up((int64_t)scan_temp_bytes(n + 1));
}

int pin_pool_window(const float* coord, int64_t n, const void* center, int32_t center_f64, double radius2,
                    int64_t tail_start, int64_t* keep, int64_t* counts, void* workspace, void* stream) {
    if (n < 0 || !center || !counts || !workspace || (n > 0 && (!coord || !keep))) return PIN_ERR_ARG;
    auto s = as_stream(stream);
    Carve c{(char*)workspace};
    int32_t* flags = c.take<int32_t>(n);
    int64_t* incl = c.take<int64_t>(n + 1);
    const size_t temp_bytes = scan_temp_bytes(n + 1);
    void* temp = c.take<char>((int64_t)temp_bytes);
    if (n > 0) {
        if (center_f64)
            hipLaunchKernelGGL(k_window_flags<double>, dim3(blocks_for(n)), dim3(kBlock), 0, s, coord, n,
                               (const double*)center, radius2, flags);
        else
            hipLaunchKernelGGL(k_window_flags<float>, dim3(blocks_for(n)), dim3(kBlock), 0, s, coord, n,
                               (const float*)center, (float)radius2, flags);
        size_t tb = temp_bytes;
        if (incl_scan(temp, tb, flags, incl, n, s) != hipSuccess) return PIN_ERR_HIP;
    }
    hipLaunchKernelGGL(k_window_write, dim3(blocks_for(n + 1)), dim3(kBlock), 0, s, flags, incl, n, tail_start, keep,
                       counts);
    return status(hipSuccess);
}

int pin_gather_rows(const PinRowArray* arrays, int32_t n_arrays, const int64_t* rows, int64_t n_rows, void* stream) {
    if (n_arrays < 0 || n_arrays > PIN_ROW_ARRAYS_MAX || n_rows < 0 || (n_arrays > 0 && !arrays)) return PIN_ERR_ARG;
    if (n_rows > 0 && !rows) return PIN_ERR_ARG;
    RowArrays A{};
    for (int a = 0; a < n_arrays; ++a) {
        const PinRowArray& x = arrays[a];
        if (x.row_bytes < 0 || (x.row_bytes > 0 && (!x.src || !x.dst))) return PIN_ERR_ARG;
        const uintptr_t align = (uintptr_t)x.src | (uintptr_t)x.dst | (uintptr_t)x.row_bytes;
        const int sh = (align & 15) == 0 ? 4 : (align & 7) == 0 ? 3 : (align & 3) == 0 ? 2 : 0;
        A.src[A.n] = (const unsigned char*)x.src;
        A.dst[A.n] = (unsigned char*)x.dst;
        A.units[A.n] = x.row_bytes >> sh;
        A.shift[A.n] = sh;
        A.n += x.row_bytes > 0 ? 1 : 0;
    }
    if (A.n == 0 || n_rows == 0) return PIN_OK;
    hipLaunchKernelGGL(k_gather_rows, dim3(blocks_for(n_rows)), dim3(kBlock), 0, as_stream(stream), A, rows, n_rows);
    return status(hipSuccess);
}

int pin_map_gather(const PinMapArrays* src, const int64_t* rows, int64_t n_rows, int32_t pad_row,
                   const PinMapArrays* dst, void* stream) {
    return move_rows(src, dst, rows, n_rows, pad_row, false, as_stream(stream));
}

int pin_map_scatter(const PinMapArrays* src, const int64_t* rows, int64_t n_rows, int32_t pad_row,
                    const PinMapArrays* dst, void* stream) {
    return move_rows(src, dst, rows, n_rows, pad_row, true, as_stream(stream));
}

int pin_map_adjust(const PinMapArrays* map, const float* pose_diff, int64_t num_poses, int32_t use_mid_ts,
                   void* stream) {
    if (!map || map->count < 0 || !pose_diff || num_poses <= 0) return PIN_ERR_ARG;
    const int64_t M = map->count;
    if (M == 0) return PIN_OK;
    if (!map->positions || !map->ts_create || (use_mid_ts && !map->ts_update)) return PIN_ERR_ARG;
    hipLaunchKernelGGL(k_map_adjust, dim3(blocks_for(M)), dim3(kBlock), 0, as_stream(stream), map->positions,
                       map->orientations, map->ts_create, map->ts_update, M, pose_diff, use_mid_ts);
    return status(hipSuccess);
}

}  // extern "C"
