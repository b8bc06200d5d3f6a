// pin_train.hip -- one mapping iteration of utils/mapper.py:443-575 as three launches.
//
//  k_train_forward   main batch (N rows) + the numerical-gradient stencil (6 * N/dec rows,
//                    generated in-kernel from coord[::dec] +- eps e_a, mapper.py:683-711):
//                    training-mode query_feature (certainty scatter_add, ts amax on the main
//                    rows, neural_points.py:637-648) + Decoder.sdf.  Saves per row the k ids,
//                    IDW weights and the decoder input x for the backward.
//  k_train_backward  dL/dsdf of  BCEWithLogits(sdf/s, sigmoid(label/s))  (loss.py:40-47) and of
//                    weight_e * mean((|g| - 1)^2) through the stencil (mapper.py:546-547);
//                    decoder backward; dL/dfeatures scattered with float atomics shaped as
//                    8 lanes x 32 B per row; optional decoder-parameter gradients.
//  k_adam            dense torch.optim.Adam step (tools.py:111-112) that also zeroes the grad.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <rocprim/block/block_radix_sort.hpp>
#include <rocprim/block/block_scan.hpp>

#include "pin_device.h"

using namespace pin;

namespace {

#ifndef PIN_TRAIN_BLOCK
#define PIN_TRAIN_BLOCK 256
#endif
constexpr int kTBlock = PIN_TRAIN_BLOCK;   // threads (rows) per block of the training kernels
static_assert(kTBlock % 64 == 0 && kTBlock <= kBlock, "training blocks are whole waves, at most kBlock threads");

inline dim3 grid_for(int64_t n) { return dim3((unsigned)((n + kTBlock - 1) / kTBlock)); }
inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline int launch_status() { return hipGetLastError() == hipSuccess ? PIN_OK : PIN_ERR_HIP; }

// Deterministic accumulation (PinTrainState.grad_fixed / cert_fixed): a float term as a 64-bit
// fixed-point integer round(v * 2^shift) (the product is exact in f64; saturated at +-2^62), added
// with integer atomics -- associative, so the sums do not depend on arrival order -- and turned
// back into a float once, after the sum.
__device__ __forceinline__ unsigned long long to_fixed(float v, double scale) {
    double t = (double)v * scale;
    t = fmin(fmax(t, -4.611686018427387904e18), 4.611686018427387904e18);
    return (unsigned long long)__double2ll_rn(t);
}
__device__ __forceinline__ float from_fixed(long long v, double inv_scale) { return (float)((double)v * inv_scale); }
__device__ __forceinline__ double fixed_scale(int shift) { return (double)(1ull << (shift & 63)); }

// The feature gradients take TWO fixed-point parts (PinTrainState.grad_fixed [2, replicas, L+1, 8]):
// a term t = g 2^shift with |t| >= 4096 goes to the coarse part as round(t); a smaller one to the
// fine part as round(t 2^40) (< 2^52: 2,048 such terms per element before any overflow).  One part
// at 2^-50 would round every term below ~4e-16 to zero and terms of ~1e-13 to a few per cent --
// and the reference's Adam (eps 1e-15) turns a gradient of 1e-18 into a step of 1e-3 lr: the
// dominated neighbours of a query that sits on a neural point (u_j / S ~ 1e-15) train on exactly
// such gradients.  Each term goes to one part, chosen by its own value, so
// the sums stay exact integers and order-free; the fold adds coarse 2^-shift + fine 2^-(shift + 40).
constexpr double kFixedFineMul = 1099511627776.0;   // 2^40
__device__ __forceinline__ void fixed_add(unsigned long long* __restrict__ dst, int64_t e, float g, double scale,
                                          int64_t fine_off) {
    const double t = (double)g * scale;
    if (fabs(t) >= 4096.0) atomicAdd(dst + e, to_fixed(g, scale));
    else if (t != 0.0) atomicAdd(dst + fine_off + e, (unsigned long long)__double2ll_rn(t * kFixedFineMul));
}
__device__ __forceinline__ float from_fixed2(long long coarse, long long fine, double inv_scale) {
    return (float)((double)coarse * inv_scale + (double)fine * (inv_scale / kFixedFineMul));
}
// offset of the fine part: the coarse part's replicas x rows x 8
__device__ __forceinline__ int64_t fixed_fine_off(const PinTrainState& st, int64_t rows) {
    return (int64_t)(st.replicas > 1 ? st.replicas : 1) * rows * kF;
}

// row r of the iteration: a main query or a stencil query (x+,x-,y+,y-,z+,z- blocks)
__device__ __forceinline__ void row_coord(const float* __restrict__ coord, const PinTrainCfg& c, int64_t r, float& qx,
                                          float& qy, float& qz) {
    if (r < c.n_main || (c.flags & PIN_TRAIN_ROWS)) {   // a batch row, or every row materialized
        qx = coord[3 * r];
        qy = coord[3 * r + 1];
        qz = coord[3 * r + 2];
        return;
    }
    const int64_t s = r - c.n_main;
    const int blk = (int)(s / c.n_stencil);
    const int64_t b = (s % c.n_stencil) * c.decimation;
    qx = coord[3 * b];
    qy = coord[3 * b + 1];
    qz = coord[3 * b + 2];
    // x + eps e_a (even blk) or x - eps e_a (odd blk), mapper.py:697-702
    if ((blk >> 1) == 0) qx = (blk & 1) ? qx - c.eps : qx + c.eps;
    else if ((blk >> 1) == 1) qy = (blk & 1) ? qy - c.eps : qy + c.eps;
    else qz = (blk & 1) ? qz - c.eps : qz + c.eps;
}

#ifndef PIN_TRAIN_FWD_MF
#define PIN_TRAIN_FWD_MF 1   // weighted_first, not PIN_TRAIN_DX, mlp->packed: the forward's sdf on the matrix cores
#endif
constexpr bool kTrainFwdMf = PIN_TRAIN_FWD_MF != 0;
#ifndef PIN_TRAIN_NWF_MF
#define PIN_TRAIN_NWF_MF 0   // 1: per-neighbour, PIN_TRAIN_DX, mlp->packed: the forward's decodes on the matrix
                             // cores (measured slower: 727 us at 2 waves/SIMD with 84 spilled VGPRs, 925 us at
                             // 1 wave, vs 644 us for the f32 VALU decodes, 1.68M rows)
#endif
constexpr bool kTrainNwfMf = PIN_TRAIN_NWF_MF != 0;
#ifndef PIN_TRAIN_NWF_WAVES
#define PIN_TRAIN_NWF_WAVES 2   // its occupancy target (the eight decodes' operands otherwise take ~340 VGPRs)
#endif
#ifndef PIN_TRAIN_NWF_NT
#define PIN_TRAIN_NWF_NT 1   // its decoder with the query tile as the outer GEMM loop (fewer live VGPRs)
#endif

#ifndef PIN_NWF_X2
#define PIN_NWF_X2 1      // per-neighbour frozen-decoder forward: two neighbours per decoder pass
#endif
#ifndef PIN_TRAIN_IDP
#define PIN_TRAIN_IDP 1   // training forward: top-k payload = feature-row id (GridSource IDP)
#endif

// MF (PIN_TRAIN_DX): whole waves call this (the matrix-core decoder); live false = a lane past
// the last row that runs slot 0 and writes nothing.  The neighbours' ids and weights are returned
// in cid / cw (-1 / 0 invalid); the block's flush_rows stores them (coalesced) and applies the
// training side effects.
template <bool WF, class Src, bool MF = false, bool DX = MF, bool PAIR = false>
__device__ __forceinline__ void train_forward_body(const Src& src, const PinPoints& p, const MlpW& m,
                                                   const float* __restrict__ coord, const int64_t* __restrict__ ts,
                                                   PinTrainCfg c, int64_t t, PinTrainState st, int (&cid)[kK],
                                                   float (&cw)[kK], bool live = true) {
    // t: processing slot (per-slot state), r: the row it processes (row order: sdf, ts)
    if (!live) t = 0;
    int64_t r;
    float qx, qy, qz;
    if (st.sorted_rows) {
        const float4 v = ((const float4*)st.sorted_rows)[t];
        qx = v.x; qy = v.y; qz = v.z;
        r = __float_as_int(v.w);
    } else {
        r = st.order ? st.order[t] : t;
        row_coord(coord, c, r, qx, qy, qz);
    }
    TopK tk;
    tk.init();
    int nn;
    if constexpr (PAIR) nn = src.template scan_pair<Src::kChunk>(qx, qy, qz, tk, threadIdx.x & 1);
    else nn = src.template scan<Src::kChunk>(qx, qy, qz, tk);
    // pair mode: both lanes of the pair hold the row's neighbours; the even lane writes its outputs
    const bool writer = live && (!PAIR || !(threadIdx.x & 1));
    const int nn_k = c.nn_k;
    resolve_ties(src, qx, qy, qz, nn_k, nn, tk);   // the reference's neighbour set at equal distances
    float u[kK];
    float S = 0.f;
#pragma unroll
    for (int j = 0; j < kK; ++j) {
        u[j] = (j < nn_k && tk.g[j] >= 0) ? 1.0f / (tk.d[j] + kIdwEps) : 0.f;
        S = S + u[j];
    }
    float x[kD];
#pragma unroll
    for (int d = 0; d < kD; ++d) x[d] = 0.f;
    float sdf = 0.f;
#if PIN_NWF_X2
    if constexpr (!WF && !MF && !PAIR && Src::kIdPayload) {
        // per-neighbour, f32 decode: neighbours j and j + 1 decoded together (mlp_sdf_packed_x2:
        // one weight read feeds both), summed in neighbour order as below; saved for the backward:
        // the ReLU masks (DX, frozen decoder) or the neighbour vectors (a training decoder)
        auto inputs = [&](int j, bool& valid, float (&xj)[kD], float& w) {
            valid = u[j] > 0.f;
            const int id = valid ? tk.g[j] : -1;
            const int64_t ii = id > 0 ? id : 0;
            float4 f0, f1;
            src.features(0, ii, f0, f1);
            float v0, v1, v2;
            if (p.positions4) {
                const float4 pp = ((const float4*)p.positions4)[ii];
                v0 = qx - pp.x;
                v1 = qy - pp.y;
                v2 = qz - pp.z;
            } else {
                v0 = qx - p.positions[3 * ii];
                v1 = qy - p.positions[3 * ii + 1];
                v2 = qz - p.positions[3 * ii + 2];
            }
            if (p.after_pgo && valid) quat_rotate_passive(((const float4*)p.orientations)[id], v0, v1, v2);
            w = valid && nn > 0 ? u[j] / S : 0.f;
            cid[j] = valid && live ? id : -1;
            cw[j] = w;
            const float xs[kD] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w, v0, v1, v2};
#pragma unroll
            for (int d = 0; d < kD; ++d) xj[d] = xs[d];
        };
#pragma unroll
        for (int j = 0; j < kK; j += 2) {
            bool va, vb;
            float xa[kD], xb[kD], wa, wb;
            inputs(j, va, xa, wa);
            inputs(j + 1, vb, xb, wb);
            float sa = 0.f, sb = 0.f;
            uint64_t ka = 0, kb = 0;
            if (va || vb) mlp_sdf_packed_x2(m, xa, xb, sa, sb, ka, kb);
            const float ska = va ? sa : 0.f, skb = vb ? sb : 0.f;
            if (!va) ka = 0;
            if (!vb) kb = 0;
            sdf = sdf + ska * wa;
            sdf = sdf + skb * wb;
            if constexpr (DX) {
                if (live && j < nn_k) ((uint2*)st.x)[t * nn_k + j] = make_uint2((uint32_t)ka, (uint32_t)(ka >> 32));
                if (live && j + 1 < nn_k)
                    ((uint2*)st.x)[t * nn_k + j + 1] = make_uint2((uint32_t)kb, (uint32_t)(kb >> 32));
            } else {
                if (live && j < nn_k) {
                    float* xo = st.x + (t * nn_k + j) * 3;
                    xo[0] = xa[kF];
                    xo[1] = xa[kF + 1];
                    xo[2] = xa[kF + 2];
                }
                if (live && j + 1 < nn_k) {
                    float* xo = st.x + (t * nn_k + j + 1) * 3;
                    xo[0] = xb[kF];
                    xo[1] = xb[kF + 1];
                    xo[2] = xb[kF + 2];
                }
            }
        }
        if (writer) st.sdf[r] = sdf;
        return;
    }
#endif
#pragma unroll
    for (int j = 0; j < kK; ++j) {
        if (j == kK / 2) __builtin_amdgcn_sched_barrier(0);
        const bool valid = u[j] > 0.f;
        int id;
        float4 f0, f1;
        float v0, v1, v2;
        if constexpr (Src::kIdPayload) {
            // payload = id: the neighbour vector reads positions[id], which is the record's position
            // bitwise for a faithful record and what the reference reads for an unfaithful one
            id = valid ? tk.g[j] : -1;
            const int64_t ii = id > 0 ? id : 0;
            src.features(0, ii, f0, f1);
            if (p.positions4) {   // one 16-B load beside the feature loads (all three by id)
                const float4 pp = ((const float4*)p.positions4)[ii];
                v0 = qx - pp.x;
                v1 = qy - pp.y;
                v2 = qz - pp.z;
            } else {
                v0 = qx - p.positions[3 * ii];
                v1 = qy - p.positions[3 * ii + 1];
                v2 = qz - p.positions[3 * ii + 2];
            }
        } else {
            const float4 rc = src.record(tk.g[j]);
            const int raw = __float_as_int(rc.w);
            id = valid ? (raw & kIdMask) : -1;
            src.features(tk.g[j], id > 0 ? id : 0, f0, f1);
            v0 = qx - rc.x;
            v1 = qy - rc.y;
            v2 = qz - rc.z;
            if (valid && (raw & PIN_RECORD_UNFAITHFUL)) {
                v0 = qx - p.positions[3 * (int64_t)id];
                v1 = qy - p.positions[3 * (int64_t)id + 1];
                v2 = qz - p.positions[3 * (int64_t)id + 2];
            }
        }
        if (p.after_pgo && valid) quat_rotate_passive(((const float4*)p.orientations)[id], v0, v1, v2);
        const float w = valid && nn > 0 ? u[j] / S : 0.f;
        const float xj[kD] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w, v0, v1, v2};
        cid[j] = valid && live ? id : -1;
        cw[j] = w;
        if (WF) {
#pragma unroll
            for (int d = 0; d < kD; ++d) x[d] = x[d] + (valid ? xj[d] : 0.f) * w;
        } else {
            float g3[3];
            float sk = 0.f;
            uint64_t mk = 0;
            if constexpr (MF) {   // per-neighbour on the matrix cores: the whole wave decodes together
                float g8[kF];
                float xz[kD];
#pragma unroll
                for (int d = 0; d < kD; ++d) xz[d] = valid ? xj[d] : 0.f;
                const float sj = mlp_sdf_mfma16<false, 0, kF, PIN_TRAIN_NWF_NT != 0>(m, xz, g8, DX ? &mk : nullptr);
                sk = valid ? sj : 0.f;
                if (!valid) mk = 0;
            } else {
                if (valid) sk = mlp_sdf<false, kF, 3>(m, xj, g3, DX ? &mk : nullptr);
            }
            sdf = sdf + sk * w;  // sum_j sdf_j w_j (mapper.py:467-468)
            if (j < nn_k && live) {
                if constexpr (DX) {
                    // PIN_TRAIN_DX, frozen decoder: the neighbour's 64 ReLU masks -- all the backward
                    // needs for its input gradient over the features (mlp_grad8_from_mask)
                    ((uint2*)st.x)[t * nn_k + j] = make_uint2((uint32_t)mk, (uint32_t)(mk >> 32));
                } else {
                    float* xo = st.x + (t * nn_k + j) * 3;  // neighbour vectors for the backward
                    xo[0] = v0;
                    xo[1] = v1;
                    xo[2] = v2;
                }
            }
        }
    }
    if (WF) {
        if constexpr (MF && !DX) {   // a training decoder: the sdf on the matrix cores, x [rows, 11] saved
            float gx[kF];
            sdf = mlp_sdf_mfma16<false, 0, kF>(m, x, gx);
            if (writer) {
#pragma unroll
                for (int d = 0; d < kD; ++d) st.x[t * kD + d] = x[d];
            }
        } else if constexpr (MF) {   // save s dsdf/dx over the features for the backward (PIN_TRAIN_DX: [rows, 8])
            float gx[kF];
            sdf = mlp_sdf_mfma16<true, 0, kF>(m, x, gx);
            if (writer) {
                float4* xo = (float4*)(st.x + t * kF);
                xo[0] = make_float4(gx[0], gx[1], gx[2], gx[3]);
                xo[1] = make_float4(gx[4], gx[5], gx[6], gx[7]);
            }
        } else {
            float gx[kD];
            sdf = mlp_sdf<false, 0, kD>(m, x, gx);
            if (writer) {
#pragma unroll
                for (int d = 0; d < kD; ++d) st.x[t * kD + d] = x[d];
            }
        }
    }
    if (writer) st.sdf[r] = sdf;
}

// End of a training forward (all lanes of every wave, each wave on its own 64 rows -- no block
// barrier): the rows' neighbour ids / weights (cid, cw) are staged in the wave's slice of the scan
// list (free once the scan and the decoder are done) and stored to st.ids / st.weights as the
// wave's contiguous [64, nn_k] run (256-B coalesced stores instead of one 4-B store per lane and
// neighbour at a 4 nn_k-B stride, which cost ~115 us of the 1.68M-row forward).  The training
// side effects are applied by the backward (train_side_effects) from these arrays.
// t0: the processing slot of the block's first row.
template <bool PAIR = false>
__device__ __forceinline__ void flush_rows(const PinTrainCfg& c, const PinTrainState& st, int64_t t0, int64_t rows,
                                           const int (&cid)[kK], const float (&cw)[kK]) {
    // pair mode: 32 rows per wave, staged by the even lanes
    constexpr int R = PAIR ? 32 : 64;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int* const s_id = wave_list();
    float* const s_w = (float*)(s_id + 64 * kK);
    static_assert(kListSeg * 64 >= 2 * 64 * kK, "flush staging must fit the wave's scan list");
    wave_lds_sync();   // the slice was the scan list / decoder scratch: every lane is past its reads
    if (!PAIR || !(lane & 1)) {
        const int lr = PAIR ? lane >> 1 : lane;
#pragma unroll
        for (int j = 0; j < kK; ++j) {
            s_id[lr * kK + j] = cid[j];
            s_w[lr * kK + j] = cw[j];
        }
    }
    wave_lds_sync();
    const int64_t tw = t0 + R * wave;   // the wave's first slot
    if (tw >= rows) return;
    const int nn_k = c.nn_k;
    const int nr = (int)(rows - tw < R ? rows - tw : R);
    int* __restrict__ ido = st.ids + tw * nn_k;
    float* __restrict__ wo = st.weights + tw * nn_k;
    if (nn_k == kK) {
        for (int e = lane; e < nr * kK; e += 64) {
            ido[e] = s_id[e];
            wo[e] = s_w[e];
        }
    } else {
        for (int e = lane; e < nr * nn_k; e += 64) {
            const int r = e / nn_k, j = e - r * nn_k;
            ido[e] = s_id[r * kK + j];
            wo[e] = s_w[r * kK + j];
        }
    }
}

template <bool WF, bool MF, bool DX = MF>
__global__ void __launch_bounds__(kTBlock)
k_train_forward_hash(const PinHash h, const PinPoints p, const PinMlp m, const float* __restrict__ coord,
                     const int64_t* __restrict__ ts, PinTrainCfg c, PinTrainState st) {
    __shared__ float s_mlp[MF ? 1 : kWSize];
    __shared__ uint4 s_pk[MF ? kPkBytes / 16 : 1];
    const MlpW mw = stage_decoder<MF>(m, s_mlp, s_pk);
    const int64_t t = xcd_block() * kTBlock + threadIdx.x;
    const int64_t rows = c.n_main + 6 * c.n_stencil;
    int cid[kK];
    float cw[kK];
#pragma unroll
    for (int j = 0; j < kK; ++j) { cid[j] = -1; cw[j] = 0.f; }
    if ((t & ~(int64_t)63) < rows) {   // whole waves (the MFMA decoder, resolve_ties); live: t < rows
        const HashSource src(h, p);
        train_forward_body<WF, HashSource, MF, DX>(src, p, mw, coord, ts, c, t, st, cid, cw, t < rows);
    }
    flush_rows(c, st, xcd_block() * kTBlock, rows, cid, cw);
}

#ifndef PIN_TRAIN_NWF_F32_WAVES
#define PIN_TRAIN_NWF_F32_WAVES 1   // the f32 per-neighbour training forward's minimum waves/SIMD (experiment switch)
#endif
#ifdef PIN_TRAIN_FWD_WAVES   // experiment: the grid training forward compiled for this many waves per SIMD
#define PIN_FWD_WAVES_ATTR __attribute__((amdgpu_waves_per_eu(PIN_TRAIN_FWD_WAVES)))
#else
#define PIN_FWD_WAVES_ATTR
#endif
// PAIR (PIN_TRAIN_PAIR, small batches): two lanes per row -- the candidate list split between
// them (GridSource::scan_pair) -- so a batch of ~1 wave per SIMD runs twice the waves with half
// the scan chain each.
template <bool WF, bool MF, bool DX = MF, bool PAIR = false>
__global__ void __launch_bounds__(kTBlock) PIN_FWD_WAVES_ATTR
__attribute__((amdgpu_waves_per_eu((!WF && MF) ? PIN_TRAIN_NWF_WAVES : (MF ? 3 : (!WF ? PIN_TRAIN_NWF_F32_WAVES : 1)))))
k_train_forward_grid(const PinGrid g, const PinPoints p, const PinMlp m, const float* __restrict__ coord,
                     const int64_t* __restrict__ ts, PinTrainCfg c, PinTrainState st) {
    __shared__ float s_mlp[MF ? 1 : kWSize];
    __shared__ uint4 s_pk[MF ? kPkBytes / 16 : 1];
    const MlpW mw = stage_decoder<MF>(m, s_mlp, s_pk);
    const int64_t tl = xcd_block() * kTBlock + threadIdx.x;   // lane slot
    const int64_t t = PAIR ? tl >> 1 : tl;                     // row slot
    const int64_t rows = c.n_main + 6 * c.n_stencil;
    int cid[kK];
    float cw[kK];
#pragma unroll
    for (int j = 0; j < kK; ++j) { cid[j] = -1; cw[j] = 0.f; }
    if ((tl & ~(int64_t)63) < (PAIR ? 2 * rows : rows)) {   // whole waves (MFMA, resolve_ties); live: t < rows
        const GridSource<false, PIN_TRAIN_IDP> src(g, p);
        train_forward_body<WF, GridSource<false, PIN_TRAIN_IDP>, MF, DX, PAIR>(src, p, mw, coord, ts, c, t, st, cid,
                                                                           cw, t < rows);
    }
    flush_rows<PAIR>(c, st, (xcd_block() * kTBlock) >> (PAIR ? 1 : 0), rows, cid, cw);
}

__global__ void __launch_bounds__(kTBlock)
k_train_rows(const float* __restrict__ coord, PinTrainCfg c, float* __restrict__ out) {
    const int64_t r = (int64_t)blockIdx.x * kTBlock + threadIdx.x;
    if (r >= c.n_main + 6 * c.n_stencil) return;
    c.flags &= ~PIN_TRAIN_ROWS;
    row_coord(coord, c, r, out[3 * r], out[3 * r + 1], out[3 * r + 2]);
}

// one thread per batch row: the row, its label and ts gathered from the pool and, for every
// decimation-th row, its six stencil rows pool[index[k*dec]] +- eps e_a (mapper.py:697-702) --
// the pool is read once per batch row
__global__ void __launch_bounds__(kTBlock)
k_train_gather(const float* __restrict__ cpool, const float* __restrict__ lpool, const int64_t* __restrict__ tpool,
               const float* __restrict__ wpool, int64_t pool_rows, const int64_t* __restrict__ index, PinTrainCfg c,
               float* __restrict__ rows, float* __restrict__ label, int64_t* __restrict__ ts,
               float* __restrict__ weight, int* __restrict__ error) {
    const int64_t r = (int64_t)blockIdx.x * kTBlock + threadIdx.x;
    if (r >= c.n_main) return;
    int64_t i = index[r];
    if (i < 0 || i >= pool_rows) {   // never gather outside the pool: clamp and report
        if (error) atomicOr(error, 1);
        i = 0;
    }
    const float qx = cpool[3 * i], qy = cpool[3 * i + 1], qz = cpool[3 * i + 2];
    const float lb = lpool[i];
    const int64_t tv = tpool ? tpool[i] : 0;
    const float wv = wpool ? fabsf(wpool[i]) : 1.f;
    rows[3 * r] = qx;
    rows[3 * r + 1] = qy;
    rows[3 * r + 2] = qz;
    label[r] = lb;
    if (tpool) ts[r] = tv;
    if (wpool) weight[r] = wv;
    if (c.n_stencil > 0 && r % c.decimation == 0 && r / c.decimation < c.n_stencil) {
        const int64_t k = r / c.decimation;
#pragma unroll
        for (int blk = 0; blk < 6; ++blk) {
            float x = qx, y = qy, z = qz;
            if ((blk >> 1) == 0) x = (blk & 1) ? x - c.eps : x + c.eps;
            else if ((blk >> 1) == 1) y = (blk & 1) ? y - c.eps : y + c.eps;
            else z = (blk & 1) ? z - c.eps : z + c.eps;
            float* o = rows + 3 * (c.n_main + blk * c.n_stencil + k);
            o[0] = x;
            o[1] = y;
            o[2] = z;
        }
    }
}

// The sample pool as one 32-B record per sample, {x, y, z, label} {ts lo, ts hi, weight, 0}, so a
// batch row costs ONE line gathered from a pool far larger than L2 instead of four (coordinates,
// label, ts, weight live in separate tensors in the reference's layout).
__global__ void __launch_bounds__(kTBlock)
k_pool_pack(const float* __restrict__ coord, const float* __restrict__ label, const int64_t* __restrict__ ts,
            const float* __restrict__ weight, int64_t n, float4* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kTBlock + threadIdx.x;
    if (i >= n) return;
    const int64_t t = ts ? ts[i] : 0;
    out[2 * i] = make_float4(coord[3 * i], coord[3 * i + 1], coord[3 * i + 2], label[i]);
    out[2 * i + 1] = make_float4(__int_as_float((int)(t & 0xffffffff)), __int_as_float((int)(t >> 32)),
                                 weight ? weight[i] : 1.f, 0.f);
}

// The batch draws of pin_train_gather_packed_draw: a counter-based generator (SplitMix64's
// finaliser over seed, iteration counter and row) in place of get_batch's two torch.randint calls
// -- row r's pool row (or new-sample slot) is uniform over [0, high) by a 64 x 64 -> high 64-bit
// multiply (bias < high / 2^64).  No draw launches, no state: the same (seed, counter) gives the
// same batch.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ int64_t batch_draw(uint64_t key, int64_t r, int64_t high) {
    return (int64_t)__umul64hi(mix64(key + (uint64_t)r * 0x9E3779B97F4A7C15ull), (uint64_t)high);
}
struct BatchDraw {
    uint64_t key;   // mix64(seed ^ mix64(counter)); 0 = take the index arrays
    int on;
};

// k_train_gather over the packed pool: the row's two 16-B halves of one 32-B record
__global__ void __launch_bounds__(kTBlock)
k_train_gather_packed(const float4* __restrict__ pool, int64_t pool_rows, const int64_t* __restrict__ index,
                      int64_t n_index, const int64_t* __restrict__ new_idx, int64_t new_count,
                      const int64_t* __restrict__ index_new, PinTrainCfg c, float* __restrict__ rows,
                      float* __restrict__ label, int64_t* __restrict__ ts, float* __restrict__ weight,
                      int* __restrict__ error, BatchDraw dr = BatchDraw{0, 0}) {
    const int64_t r = (int64_t)blockIdx.x * kTBlock + threadIdx.x;
    if (r >= c.n_main) return;
    int64_t i;
    if (r < n_index) {
        i = dr.on ? batch_draw(dr.key, r, pool_rows) : index[r];
    } else {   // get_batch's new-sample rows: new_idx[index_new[.]] (utils/mapper.py:335-340)
        int64_t j = dr.on ? batch_draw(dr.key, r, new_count) : index_new[r - n_index];
        if (j < 0 || j >= new_count) {
            if (error) atomicOr(error, 1);
            j = 0;
        }
        i = new_idx[j];
    }
    if (i < 0 || i >= pool_rows) {   // never gather outside the pool: clamp and report
        if (error) atomicOr(error, 1);
        i = 0;
    }
    const float4 a = pool[2 * i], b = pool[2 * i + 1];
    rows[3 * r] = a.x;
    rows[3 * r + 1] = a.y;
    rows[3 * r + 2] = a.z;
    label[r] = a.w;
    if (ts) ts[r] = (int64_t)(uint32_t)__float_as_int(b.x) | ((int64_t)__float_as_int(b.y) << 32);
    if (weight) weight[r] = fabsf(b.z);
    if (c.n_stencil > 0 && r % c.decimation == 0 && r / c.decimation < c.n_stencil) {
        const int64_t k = r / c.decimation;
#pragma unroll
        for (int blk = 0; blk < 6; ++blk) {
            float x = a.x, y = a.y, z = a.z;
            if ((blk >> 1) == 0) x = (blk & 1) ? x - c.eps : x + c.eps;
            else if ((blk >> 1) == 1) y = (blk & 1) ? y - c.eps : y + c.eps;
            else z = (blk & 1) ? z - c.eps : z + c.eps;
            float* o = rows + 3 * (c.n_main + blk * c.n_stencil + k);
            o[0] = x;
            o[1] = y;
            o[2] = z;
        }
    }
}

__device__ __forceinline__ float sigmoidf_(float v) { return 1.f / (1.f + expf(-v)); }

// loss / gradient factor of a batch row: grad_scale, or grad_scale_tail for the last n_tail rows
__device__ __forceinline__ float main_row_scale(const PinTrainCfg& c, int64_t r) {
    return r >= c.n_main - c.n_tail ? c.grad_scale_tail : c.grad_scale;
}

// the same for any row: a stencil row takes its group's base row (coord[k * decimation])
__device__ __forceinline__ float row_scale(const PinTrainCfg& c, int64_t r) {
    if (r < c.n_main) return main_row_scale(c, r);
    const int64_t k = (r - c.n_main) % c.n_stencil;
    return main_row_scale(c, k * c.decimation);
}

// dL/dsdf of row r and its loss term, unscaled (BCE rows: mean over N, weighted by the row's
// |weight| under loss_weight_on, loss.py:40-47; stencil groups: weight_e * mean over N/dec)
__device__ __forceinline__ float row_dsdf(const PinTrainCfg& c, const float* __restrict__ sdf,
                                          const float* __restrict__ label, const float* __restrict__ rw, int64_t r,
                                          double& loss) {
    loss = 0.0;
    if (r < c.n_main) {
        const float pz = sdf[r] / c.sigma;
        const float y = sigmoidf_(label[r] / c.sigma);
        const float wr = rw ? rw[r] : 1.f;
        loss = (double)fmaxf(pz, 0.f) - (double)pz * y + log1p(exp(-fabs((double)pz)));
        loss *= (double)wr / (double)c.n_main;
        return wr * (sigmoidf_(pz) - y) / ((float)c.n_main * c.sigma);
    }
    const int64_t s = r - c.n_main;
    const int blk = (int)(s / c.n_stencil);
    const int64_t k = s % c.n_stencil;
    const float* g6 = sdf + c.n_main + k;
    const float two_eps = 2.f * c.eps;
    const float gv[3] = {(g6[0] - g6[c.n_stencil]) / two_eps, (g6[2 * c.n_stencil] - g6[3 * c.n_stencil]) / two_eps,
                         (g6[4 * c.n_stencil] - g6[5 * c.n_stencil]) / two_eps};
    const float gn = sqrtf((gv[0] * gv[0] + gv[1] * gv[1]) + gv[2] * gv[2]);
    if (blk == 0) loss = c.weight_e * (double)(gn - 1.f) * (gn - 1.f) / (double)c.n_stencil;
    const float dg = c.weight_e * 2.f * (gn - 1.f) / (gn > 0.f ? gn : 1.f) / (float)c.n_stencil;
    const float d_axis = dg * gv[blk >> 1] / two_eps;
    return (blk & 1) ? -d_axis : d_axis;
}

// ------------------------------------------------------------------ analytic-gradient eikonal
// numerical_grad off (utils/mapper.py:50-54, :481-482): g = dsdf/dq by autograd with
// create_graph=True (utils/tools.py:174-184) and the eikonal term weight_e * mean((|g| - 1)^2)
// over the batch, backpropagated through g -- a double backward.  Closed form, per row, with the
// neighbour weights w_j = u_j / S, u_j = 1 / (d_j^2 + eps), c_j = du_j/dq / S = -2 u_j^2 (q - p_j) / S
// (so dw_j/dq = c_j - w_j C, C = sum_j c_j):
//   weighted_first:  g = J^T gx - (gx . x) C + Wr gx[8:],  J = sum_j x_j (x) c_j,  Wr = sum_j w_j R_j
//   per-neighbour:   g = sum_j s_j c_j - sdf C + sum_j w_j R_j gx_j[8:]
// (R_j the point's rotation after PGO, else I; gx = dsdf/dx of the decoder, which depends on the
// features / parameters only through x and the ReLU mask, whose derivative is 0).  With
// u = dL/dg = weight_e (|g| - 1) 2 g / (|g| N) (0 at |g| = 0, torch's norm backward) and
// alpha_j = u . (c_j - w_j C):
//   dL/df_j   = alpha_j gx[0:8]                         (weighted_first; gx_j[0:8] per-neighbour)
//   dL/dtheta = through gx (W1, w2; b1 and b2 only through the mask):
//     weighted_first: dL/dgx = r = J u - (u . C) x + [0, Wr^T u]
//     per-neighbour:  dL/ds_j += alpha_j, dL/dgx_j[8:] = w_j R_j^T u
// The forward writes alpha_j per slot (eik_coef) and r / u plus the row's eikonal loss (eik_vec);
// the backward adds them to the BCE terms.
constexpr int kEikWf = 20;    // eik_vec row, weighted_first: r[0..10], loss, gx[0..7]
constexpr int kEikNwf = 4;    // eik_vec row, per-neighbour: u[0..2], loss

template <bool WF, class Src>
__device__ __forceinline__ void train_forward_eik_body(const Src& src, const PinPoints& p, const MlpW& m,
                                                       const float* __restrict__ coord,
                                                       const int64_t* __restrict__ ts, const PinTrainCfg& c,
                                                       int64_t t, const PinTrainState& st, bool mlp_trains) {
    int64_t r;
    float qx, qy, qz;
    if (st.sorted_rows) {
        const float4 v = ((const float4*)st.sorted_rows)[t];
        qx = v.x; qy = v.y; qz = v.z;
        r = __float_as_int(v.w);
    } else {
        r = st.order ? st.order[t] : t;
        row_coord(coord, c, r, qx, qy, qz);
    }
    TopK tk;
    tk.init();
    const int nn = src.template scan<Src::kChunk>(qx, qy, qz, tk);
    const int nn_k = c.nn_k;
    resolve_ties(src, qx, qy, qz, nn_k, nn, tk);   // the reference's neighbour set at equal distances
    float u[kK];
    float S = 0.f;
#pragma unroll
    for (int j = 0; j < kK; ++j) {
        u[j] = (j < nn_k && tk.g[j] >= 0) ? 1.0f / (tk.d[j] + kIdwEps) : 0.f;
        S = S + u[j];
    }
    const float invS = nn > 0 ? 1.f / S : 0.f;
    float x[kD], J[kD][3], C[3] = {0.f, 0.f, 0.f}, Wr[3][3], cc[kK][3], cw[kK];
    float A[3] = {0.f, 0.f, 0.f}, G[3] = {0.f, 0.f, 0.f}, sdf = 0.f;
#pragma unroll
    for (int d = 0; d < kD; ++d) { x[d] = 0.f; J[d][0] = J[d][1] = J[d][2] = 0.f; }
#pragma unroll
    for (int a = 0; a < 3; ++a) Wr[a][0] = Wr[a][1] = Wr[a][2] = 0.f;
#pragma unroll
    for (int j = 0; j < kK; ++j) {
        const bool valid = u[j] > 0.f;
        const float4 rc = src.record(tk.g[j]);
        const int raw = __float_as_int(rc.w);
        const int id = valid ? (raw & kIdMask) : -1;
        const int64_t ii = id > 0 ? id : 0;
        float4 f0, f1;
        src.features(tk.g[j], ii, f0, f1);
        const float pg[3] = {qx - rc.x, qy - rc.y, qz - rc.z};   // the distance's (global) position
        float v0 = pg[0], v1 = pg[1], v2 = pg[2];
        if (valid && (raw & PIN_RECORD_UNFAITHFUL)) {
            v0 = qx - p.positions[3 * ii];
            v1 = qy - p.positions[3 * ii + 1];
            v2 = qz - p.positions[3 * ii + 2];
        }
        float4 qt = make_float4(1.f, 0.f, 0.f, 0.f);
        if (p.after_pgo && valid) {
            qt = ((const float4*)p.orientations)[ii];
            quat_rotate_passive(qt, v0, v1, v2);
        }
        const float w = valid && nn > 0 ? u[j] / S : 0.f;
        const float xj[kD] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w, v0, v1, v2};
        if (j < nn_k) {
            st.ids[t * nn_k + j] = id;
            st.weights[t * nn_k + j] = w;
        }
        cw[j] = w;
        const float cu = valid ? -2.f * u[j] * u[j] * invS : 0.f;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            cc[j][a] = cu * pg[a];
            C[a] += cc[j][a];
        }
        float R[3][3];
        quat_rotmat(qt, R);
        if (WF) {
#pragma unroll
            for (int d = 0; d < kD; ++d) {
                const float xv = valid ? xj[d] : 0.f;
                x[d] = x[d] + xv * w;
#pragma unroll
                for (int a = 0; a < 3; ++a) J[d][a] = fmaf(xv, cc[j][a], J[d][a]);
            }
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = 0; b < 3; ++b) Wr[a][b] = fmaf(w, R[a][b], Wr[a][b]);
        } else {
            float g3[3] = {0.f, 0.f, 0.f};
            float sk = 0.f;
            if (valid) sk = mlp_sdf<true, kF, 3>(m, xj, g3);
            sdf = sdf + sk * w;   // sum_j sdf_j w_j (mapper.py:467-468)
            float r0, r1, r2;
            quat_rotate_active(qt, g3[0], g3[1], g3[2], r0, r1, r2);
            G[0] = fmaf(w, r0, G[0]);
            G[1] = fmaf(w, r1, G[1]);
            G[2] = fmaf(w, r2, G[2]);
#pragma unroll
            for (int a = 0; a < 3; ++a) A[a] = fmaf(sk, cc[j][a], A[a]);
            if (j < nn_k) {
                float* xo = st.x + (t * nn_k + j) * 3;   // neighbour vectors for the backward
                xo[0] = v0;
                xo[1] = v1;
                xo[2] = v2;
            }
        }
    }
    float g[3] = {0.f, 0.f, 0.f};
    float gx[kD];
    if (WF) {
        sdf = mlp_sdf<true, 0, kD>(m, x, gx);
        if (nn > 0) {
            float abar = 0.f;
#pragma unroll
            for (int d = 0; d < kD; ++d) abar = fmaf(gx[d], x[d], abar);
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                float s = -abar * C[a];
#pragma unroll
                for (int d = 0; d < kD; ++d) s = fmaf(gx[d], J[d][a], s);
#pragma unroll
                for (int b = 0; b < 3; ++b) s = fmaf(Wr[a][b], gx[kF + b], s);
                g[a] = s;
            }
        }
    } else if (nn > 0) {
#pragma unroll
        for (int a = 0; a < 3; ++a) g[a] = A[a] - sdf * C[a] + G[a];
    }
    // eikonal term of this row: weight_e (|g| - 1)^2 / N, scaled like the row's BCE term
    const float gn = sqrtf((g[0] * g[0] + g[1] * g[1]) + g[2] * g[2]);
    const float rs = main_row_scale(c, r);
    const float cu = gn > 0.f ? c.weight_e * rs * 2.f * (gn - 1.f) / (gn * (float)c.n_main) : 0.f;
    const float uq[3] = {cu * g[0], cu * g[1], cu * g[2]};
    const float loss = c.weight_e * rs * (gn - 1.f) * (gn - 1.f) / (float)c.n_main;
    const float uC = (uq[0] * C[0] + uq[1] * C[1]) + uq[2] * C[2];
#pragma unroll
    for (int j = 0; j < kK; ++j) {
        if (j >= nn_k) break;
        const float al = (uq[0] * cc[j][0] + uq[1] * cc[j][1]) + uq[2] * cc[j][2] - cw[j] * uC;
        st.eik_coef[t * nn_k + j] = al;
    }
    if (WF) {
        float* ev = st.eik_vec + t * kEikWf;
#pragma unroll
        for (int d = 0; d < kD; ++d) st.x[t * kD + d] = x[d];
#pragma unroll
        for (int d = 0; d < kF; ++d) ev[12 + d] = gx[d];
        ev[11] = loss;
        if (mlp_trains) {
#pragma unroll
            for (int d = 0; d < kD; ++d) {
                float rv = -uC * x[d];
#pragma unroll
                for (int a = 0; a < 3; ++a) rv = fmaf(J[d][a], uq[a], rv);
                if (d >= kF) {
#pragma unroll
                    for (int a = 0; a < 3; ++a) rv = fmaf(Wr[a][d - kF], uq[a], rv);
                }
                ev[d] = rv;
            }
        }
    } else {
        float* ev = st.eik_vec + t * kEikNwf;
        ev[0] = uq[0];
        ev[1] = uq[1];
        ev[2] = uq[2];
        ev[3] = loss;
    }
    st.sdf[r] = sdf;
}

template <bool WF, class Src>
__device__ __forceinline__ void train_forward_eik_kernel_body(const Src& src, const PinPoints& p, const MlpW& mw,
                                                              const float* coord, const int64_t* ts, PinTrainCfg c,
                                                              PinTrainState st, bool mlp_trains) {
    const int64_t t = xcd_block() * kTBlock + threadIdx.x;
    // whole waves (resolve_ties): lanes past the rows redo the last row (identical values to the
    // same addresses; this forward has no atomics)
    if ((t & ~(int64_t)63) < c.n_main)
        train_forward_eik_body<WF>(src, p, mw, coord, ts, c, t < c.n_main ? t : c.n_main - 1, st, mlp_trains);
}

template <bool WF>
__global__ void __launch_bounds__(kTBlock)
k_train_forward_eik_hash(const PinHash h, const PinPoints p, const PinMlp m, const float* __restrict__ coord,
                         const int64_t* __restrict__ ts, PinTrainCfg c, PinTrainState st, int mlp_trains) {
    __shared__ float s_mlp[kWSize];
    const MlpW mw = stage_mlp(m, s_mlp);
    train_forward_eik_kernel_body<WF>(HashSource(h, p), p, mw, coord, ts, c, st, mlp_trains != 0);
}

template <bool WF>
__global__ void __launch_bounds__(kTBlock)
k_train_forward_eik_grid(const PinGrid g, const PinPoints p, const PinMlp m, const float* __restrict__ coord,
                         const int64_t* __restrict__ ts, PinTrainCfg c, PinTrainState st, int mlp_trains) {
    __shared__ float s_mlp[kWSize];
    const MlpW mw = stage_mlp(m, s_mlp);
    train_forward_eik_kernel_body<WF>(GridSource<false, false>(g, p), p, mw, coord, ts, c, st, mlp_trains != 0);
}

// The training side effects of the iteration's training-mode query (neural_points.py:640
// certainty scatter_add of the IDW weights, :644 ts_update amax with the batch rows' ts), applied
// at the end of the backward from the saved ids / weights (all threads of the block):
//  1. every (row, neighbour) of the block's rows writes its id as the tag of slot id & (S-1) of
//     an LDS table; after a barrier the pairs whose id kept the slot add their weight (LDS float
//     add) and max their row's ts (LDS int max) into it -- no returning atomics -- and a pair
//     whose slot went to another id goes to memory directly;
//  2. the table goes out slot by slot: one memory-side atomic (and one ts_update read) per
//     distinct point of the block, each instruction covering consecutive slots, i.e. ids that
//     differ in their low bits only.
// In the forward, one atomic per (row, neighbour) pair scattered over the rows' neighbourhoods
// cost ~115 us of the 1.68M-row iteration (the same atomics at contiguous addresses: ~17 us).
constexpr int kCertSlots = 4 * kTBlock;   // 1,024 slots for the 256-row block's <= 2,048 pairs

__device__ __forceinline__ void ts_amax(int64_t* __restrict__ ts_update, int id, int64_t q) {
    if (ts_update[id] < q) atomicMax((unsigned long long*)(ts_update + id), (unsigned long long)q);
}

constexpr int kSideBufInts = 3 * kCertSlots + 2 * kTBlock;   // tag, val, ts per slot + the rows' int64 ts

// The table in buf (kSideBufInts ints of the block's LDS): tag, weight sum and max ts per slot,
// then the block's rows' ts.
struct SideTable {
    int* tag;
    float* val;
    int* ts;
    int64_t* rts;
    float* cert;                 // float certainty sums (NULL in the deterministic mode)
    unsigned long long* cfix;    // deterministic mode: fixed-point certainty sums, one atomic per pair
    double cscale;
    int64_t* ts_update;
    __device__ SideTable(int* buf, const PinTrainState& st)
        : tag(buf), val((float*)(buf + kCertSlots)), ts(buf + 2 * kCertSlots), rts((int64_t*)(buf + 3 * kCertSlots)),
          cert(st.cert_fixed ? nullptr : st.certainties), cfix((unsigned long long*)st.cert_fixed),
          cscale(fixed_scale(st.cert_shift)), ts_update(st.row_ts ? st.ts_update : nullptr) {}
    // all threads, then a barrier before any claim: empty slots; thread tid's row ts (batch rows
    // only -- the stencil rows' query carries none)
    __device__ void init(const PinTrainCfg& c, const PinTrainState& st, int nrow_blk, int64_t row) const {
        const int tid = threadIdx.x;
        rts[tid] = (ts_update && tid < nrow_blk && row < c.n_main) ? st.row_ts[row] : -1;
        for (int k = tid; k < kCertSlots; k += kTBlock) {
            tag[k] = -1;
            val[k] = 0.f;
            ts[k] = -1;
        }
    }
    __device__ void claim(int id) const {
        if (id >= 0) tag[id & (kCertSlots - 1)] = id;
    }
    // after a barrier that follows every claim: pair (id, w) of local row lr
    __device__ void add(int id, float w, int lr) const {
        if (id < 0) return;
        if (cfix) atomicAdd(cfix + id, to_fixed(w, cscale));
        const int k = id & (kCertSlots - 1);
        const int64_t q = rts[lr];
        if (tag[k] == id && q <= 0x7fffffff) {
            if (cert) atomicAdd(val + k, w);
            if (q >= 0) atomicMax(ts + k, (int)q);
        } else {   // the slot went to another id (or a ts beyond int32): straight to memory
            if (cert) atomicAdd(cert + id, w);
            if (ts_update && q >= 0) ts_amax(ts_update, id, q);
        }
    }
    // after a barrier that follows every add: one memory-side atomic per occupied slot
    __device__ void flush() const {
        for (int k = threadIdx.x; k < kCertSlots; k += kTBlock) {
            const int id = tag[k];
            if (id < 0) continue;
            if (cert) atomicAdd(cert + id, val[k]);
            if (ts_update && ts[k] >= 0) ts_amax(ts_update, id, ts[k]);
        }
    }
};

// The side effects on their own (no feature scatter to ride on): the block's ids / weights read
// from memory.  All threads.
__device__ __forceinline__ void train_side_effects(const PinTrainCfg& c, const PinTrainState& st, int64_t row0,
                                                   int nrow_blk, int64_t row, int* buf) {
    const SideTable tb(buf, st);
    const int nn_k = c.nn_k;
    const int npair = nrow_blk * nn_k;   // <= kTBlock * kK: kK pairs per thread, held in registers
    const int* __restrict__ ids = st.ids + row0 * nn_k;
    const float* __restrict__ ws = st.weights + row0 * nn_k;
    int pid[kK];
    float pw[kK];
#pragma unroll
    for (int u = 0; u < kK; ++u) {
        const int e = threadIdx.x + u * kTBlock;
        pid[u] = e < npair ? ids[e] : -1;
        pw[u] = e < npair ? ws[e] : 0.f;
    }
    tb.init(c, st, nrow_blk, row);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kK; ++u) tb.claim(pid[u]);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kK; ++u) tb.add(pid[u], pw[u], (threadIdx.x + u * kTBlock) / nn_k);
    __syncthreads();
    tb.flush();
}

// backward: one row per lane for the decoder; the row's k x 8 feature-gradient terms are staged
// in LDS and scattered with 64 lanes covering 8 rows x 32 contiguous bytes per instruction.
// Decoder-parameter gradients (a training decoder): GEMMs over the rows on the f32 matrix cores
// (mlp_grad_mfma) -> per-block partials (fixed order, no same-address atomics) ->
// k_mlp_grad_final, which also turns the reduced products into dW1, db1, dW2, db2.
constexpr int kMlpGrad = PIN_MLP_GRAD_SIZE;
constexpr int kWaves = kTBlock / 64;
constexpr int kTSize = kH * 16;                 // T[c][i], i < 16 (12 used)
constexpr int kMlpPart = PIN_MLP_PART_FLOATS;   // per block: T, T' (analytic eikonal), sum so
static_assert(kMlpPart >= 2 * kTSize + 1, "decoder-gradient partial layout");
constexpr int kMgWave = 128 + 2 * 1024;         // per-wave LDS of mlp_grad_mfma: masks, B, E

__device__ __forceinline__ float wave_sum_f(float v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// decoder backward of one input row x with upstream dL/d(out) = so (already times sdf_scale):
// gf += sum_c delta_c W1[c][0:8], delta_c = so w2_c 1[pre_c > 0].  Returns the row's 64 ReLU
// masks (bit c) for the decoder-parameter products (mlp_grad_mfma).
__device__ __forceinline__ uint64_t decoder_backward_row(const MlpW& m, const float (&x)[kD], float so,
                                                         float (&gf)[kF]) {
    uint32_t lo = 0u, hi = 0u;
#pragma unroll 2
    for (int cc = 0; cc < kH; ++cc) {
        float wr[kWRow];
        load_row(m.w, cc, wr);
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < kD; ++i) acc = fmaf(wr[i], x[i], acc);
        const float pre = acc + m.w[kWB1 + cc];
        const bool on = pre > 0.f;
        const float delta = on ? so * m.w[kWW2 + cc] : 0.f;
#pragma unroll
        for (int d = 0; d < kF; ++d) gf[d] = fmaf(delta, wr[d], gf[d]);
        const uint32_t bit = on ? 1u << (cc & 31) : 0u;
        if (cc < 32) lo |= bit; else hi |= bit;
    }
    return ((uint64_t)hi << 32) | lo;
}

// The decoder-parameter gradients of the wave's 64 rows (one lane per row) as products over the
// rows, accumulated on v_mfma_f32_16x16x4_f32 (exact f32 products, f32 sums):
//   T[c][i]  += sum_r 1[pre_c(r) > 0] so(r) [x(r), 1]_i        (i < 12)
//   T'[c][i] += sum_r 1[pre_c(r) > 0] e_i(r)                    (EXTRA: the analytic eikonal's
//                                                                dL/d(gx) of each row, gx = s W1^T (w2 o 1))
// from which k_mlp_grad_final forms dW1[c][i] = w2_c (T + s T')[c][i], db1_c = w2_c T[c][11],
// dW2_c = W1[c] . (T + s T')[c][0:11] + b1_c T[c][11].  A = the 0/1 masks (hidden c x row), B =
// the rows' values (row x i), staged through the wave's LDS slice ws (kMgWave floats) transposed
// so that a lane's 16 k-steps (rows 4 ks + g) are contiguous.  Every lane of the wave calls this.
template <bool EXTRA>
__device__ __forceinline__ void mlp_grad_mfma(float* ws, uint64_t mask, float so, const float (&x)[kD],
                                              const float* e, f32x4 (&accT)[4], f32x4 (&accE)[4]) {
    const int lane = threadIdx.x & 63;
    const int slot = (lane & 3) * 16 + (lane >> 2);   // row r -> [g = r & 3][ks = r >> 2]
    uint32_t* wm = (uint32_t*)ws;                      // [2 halves][64]
    float* wb = ws + 128;                              // [16 i][64]
    float* we = ws + 128 + 1024;                       // [16 i][64]
    wave_lds_sync();   // the previous call's readers are done
    wm[slot] = (uint32_t)mask;
    wm[64 + slot] = (uint32_t)(mask >> 32);
#pragma unroll
    for (int i = 0; i < kD; ++i) wb[i * 64 + slot] = so * x[i];
    wb[kD * 64 + slot] = so;
#pragma unroll
    for (int i = kD + 1; i < 16; ++i) wb[i * 64 + slot] = 0.f;
    if (EXTRA) {
#pragma unroll
        for (int i = 0; i < kD; ++i) we[i * 64 + slot] = e[i];
#pragma unroll
        for (int i = kD; i < 16; ++i) we[i * 64 + slot] = 0.f;
    }
    wave_lds_sync();
    const int n = lane & 15, g = lane >> 4;
#pragma unroll
    for (int kq = 0; kq < 4; ++kq) {
        const float4 b4 = *(const float4*)(wb + n * 64 + g * 16 + 4 * kq);
        const uint4 lo4 = *(const uint4*)(wm + g * 16 + 4 * kq);
        const uint4 hi4 = *(const uint4*)(wm + 64 + g * 16 + 4 * kq);
        float4 e4 = make_float4(0.f, 0.f, 0.f, 0.f);
        if (EXTRA) e4 = *(const float4*)(we + n * 64 + g * 16 + 4 * kq);
        const float bv[4] = {b4.x, b4.y, b4.z, b4.w};
        const float ev[4] = {e4.x, e4.y, e4.z, e4.w};
        const uint32_t lv[4] = {lo4.x, lo4.y, lo4.z, lo4.w};
        const uint32_t hv[4] = {hi4.x, hi4.y, hi4.z, hi4.w};
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
            for (int ct = 0; ct < 4; ++ct) {
                const uint32_t w = ct < 2 ? lv[s] : hv[s];
                const float a = (float)((w >> ((16 * ct + n) & 31)) & 1u);
                accT[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv[s], accT[ct], 0, 0, 0);
                if (EXTRA) accE[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, ev[s], accE[ct], 0, 0, 0);
            }
        }
    }
}

// End of the block: the waves' T (T') and sum so into the block's partial (fixed order).
// s_mg: [kWaves][kMgWave]; all threads call this.
template <bool EXTRA>
__device__ __forceinline__ void mlp_grad_flush(float (*s_mg)[kMgWave], float* s_so, const f32x4 (&accT)[4],
                                               const f32x4 (&accE)[4], float so_sum, float* __restrict__ part) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n = lane & 15, g = lane >> 4;
    const float s = wave_sum_f(so_sum);
    wave_lds_sync();
    float* tw = s_mg[wave] + 128;
#pragma unroll
    for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = 16 * ct + 4 * g + j;   // accumulator row -> hidden unit, column -> i
            tw[c * 16 + n] = accT[ct][j];
            if (EXTRA) tw[kTSize + c * 16 + n] = accE[ct][j];
        }
    if (lane == 0) s_so[wave] = s;
    __syncthreads();
    constexpr int nval = EXTRA ? 2 * kTSize : kTSize;
    for (int e = threadIdx.x; e < nval; e += kTBlock) {
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) v += s_mg[w][128 + e];
        part[e] = v;
    }
    if (threadIdx.x == 0) {
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) v += s_so[w];
        part[2 * kTSize] = v;
    }
}

// decoder backward of one input row x with upstream dL/d(out) = so (already times sdf_scale),
// frozen decoder: gf += sum_c delta_c W1[c][0:8]
__device__ __forceinline__ void decoder_backward(const MlpW& m, const float (&x)[kD], float so, float (&gf)[kF]) {
#pragma unroll 2
    for (int cc = 0; cc < kH; ++cc) {
        float wr[kWRow];
        load_row(m.w, cc, wr);
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < kD; ++i) acc = fmaf(wr[i], x[i], acc);
        const float pre = acc + m.w[kWB1 + cc];
        const float delta = pre > 0.f ? so * m.w[kWW2 + cc] : 0.f;
#pragma unroll
        for (int d = 0; d < kF; ++d) gf[d] = fmaf(delta, wr[d], gf[d]);
    }
}

#ifndef PIN_SCAT_UNROLL
#define PIN_SCAT_UNROLL 1
#endif

// Scatter of the block's weighted_first feature-gradient rows (all threads; after a barrier):
// element e = (row, j, d), d fastest: a wave instruction covers 8 (row, neighbour) pairs x 32
// contiguous bytes, one memory-side request each -- the cheapest atomic shape measured (LDS
// pre-aggregation per block, and 64-B rows carrying the certainty, were slower).  The block's ids
// and weights are staged in LDS first with coalesced loads, so the scatter loop issues its
// atomics back to back instead of waiting on a load per element.
// buf: (2 + EIK) kTBlock kK ints of the block's LDS
template <bool EIK>
__device__ __forceinline__ void feature_scatter(const PinTrainCfg& c, const PinTrainState& st, int64_t row0,
                                                int nrow_blk, const float* gst, const float* s_dsdf,
                                                float* __restrict__ grad_features, unsigned long long* __restrict__ fdst,
                                                double fscale, int* buf, int64_t frows = 1) {
    const int64_t ffine = fixed_fine_off(st, frows);
    int* const s_ids = buf;
    float* const s_wt = (float*)(buf + kTBlock * kK);
    float* const s_al = (float*)(buf + 2 * kTBlock * kK);
    const int nn_k = c.nn_k;
    const int npair = nrow_blk * nn_k;
    for (int e = threadIdx.x; e < npair; e += kTBlock) {
        s_ids[e] = st.ids[row0 * nn_k + e];
        s_wt[e] = st.weights[row0 * nn_k + e];
        if (EIK) s_al[e] = st.eik_coef[row0 * nn_k + e];
    }
    __syncthreads();
    const int total = npair * kF;
#pragma unroll PIN_SCAT_UNROLL
    for (int e = threadIdx.x; e < total; e += kTBlock) {
        const int d = e & (kF - 1);
        const int rj = e >> 3;
#if defined(PIN_EXP_SCAT2) && PIN_EXP_SCAT2 == 1   // timing variant: contiguous rows (wrong sums)
        const int id = s_ids[rj] < 0 ? -1 : (int)((row0 * nn_k + rj) % frows);
#elif defined(PIN_EXP_SCAT2) && PIN_EXP_SCAT2 == 2   // timing variant: the block's pairs onto one point (wrong sums)
        const int id = s_ids[rj] < 0 ? -1 : (int)(blockIdx.x % frows);
#else
        const int id = s_ids[rj];
#endif
        if (id < 0) continue;
        const int lr = rj / nn_k;
        float g;
        if (EIK) g = fmaf(s_wt[rj], s_dsdf[lr], s_al[rj]) * gst[lr * kF + d];
        else g = s_wt[rj] * gst[lr * kF + d];
        if (fdst) fixed_add(fdst, (int64_t)id * kF + d, g, fscale, ffine);   // deterministic mode
        else atomicAdd(grad_features + (int64_t)id * kF + d, g);
    }
}


#ifndef PIN_SCAT_SORT
#define PIN_SCAT_SORT 1   // 0: the unsorted scatter for every batch (A/B builds)
#endif
#ifndef PIN_NWF_SORT
#define PIN_NWF_SORT 1    // 0: the per-neighbour mask backward scatters per wave, unsorted (A/B builds)
#endif
// the per-neighbour mask path reads the ReLU masks the forward's f32 decode saves: the row-wise
// experiment decoder (mlp_sdf_rows) does not produce them
static_assert(PIN_MLP_ROWS == 0, "PIN_MLP_ROWS builds lack the ReLU masks of the PIN_TRAIN_DX per-neighbour path");

// The same scatter with the block's (row, neighbour) pairs pre-summed per feature row: the pairs
// are radix-sorted by id in LDS (rocprim block sort, ceil(log2 rows) bits, stable), each run of
// equal ids becomes one 32-B row of float atomics (8 lanes x 32 contiguous bytes per run, the
// shape above) -- the memory-side atomics fall by the block's references per row (~2-3 on
// tile-sorted rows), at the cost of the sort.  Runs are summed in sorted (= input) order.
// side: the training side effects ride on the same runs (train_side_effects' semantics): per run
// one certainty add of its weights' sum (fixed-point: the sum of the pairs' fixed-point values)
// and one ts max over its batch rows' ts.  row: the calling thread's row (its ts).
template <bool EIK = false>
__device__ __forceinline__ void feature_scatter_sorted(const PinTrainCfg& c, const PinTrainState& st, int64_t row0,
                                                       int nrow_blk, const float* gst, const float* s_dsdf,
                                                       float* __restrict__ grad_features,
                                                       unsigned long long* __restrict__ fdst, double fscale,
                                                       int* buf, int64_t frows, bool side, int64_t row) {
    constexpr int kP = kTBlock * kK;
    using Sort = rocprim::block_radix_sort<unsigned, kTBlock, kK, unsigned short>;
    using Scan = rocprim::block_scan<int, kTBlock>;
    __shared__ union {
        typename Sort::storage_type sort;
        typename Scan::storage_type scan;
    } s_tmp;
    __shared__ unsigned short s_val[kP];        // sorted position -> pair index
    __shared__ int s_run_id[kP];
    __shared__ unsigned short s_run_start[kP];
    __shared__ unsigned s_last[kTBlock];
    __shared__ int64_t s_rts[kTBlock];           // the block's rows' ts (side effects)
    __shared__ int s_end;                        // sorted position of the first invalid pair
    int* const s_ids = buf;
    float* const s_wt = (float*)(buf + kTBlock * kK);
    float* const s_al = (float*)(buf + 2 * kTBlock * kK);   // EIK: the pairs' eik_coef
    const int nn_k = c.nn_k;
    const int npair = nrow_blk * nn_k;
    for (int e = threadIdx.x; e < npair; e += kTBlock) {
        s_ids[e] = st.ids[row0 * nn_k + e];
        s_wt[e] = st.weights[row0 * nn_k + e];
        if (EIK) s_al[e] = st.eik_coef[row0 * nn_k + e];
    }
    if (threadIdx.x == 0) s_end = kP;
    int64_t* const ts_update = (side && st.row_ts) ? st.ts_update : nullptr;
    if (side)
        s_rts[threadIdx.x] = (ts_update && (int)threadIdx.x < nrow_blk && row < c.n_main) ? st.row_ts[row] : -1;
    __syncthreads();
    // 2^bits > frows > any id (ids are int32 row indices; 32 bits when frows needs them all)
    const unsigned bits = frows >= (int64_t)0x80000000u ? 32u : 32u - (unsigned)__clz((unsigned)frows);
    const unsigned inval = bits >= 32u ? ~0u : (1u << bits) - 1u;
    unsigned keys[kK];
    unsigned short vals[kK];
#pragma unroll
    for (int i = 0; i < kK; ++i) {
        const int pidx = threadIdx.x * kK + i;
        const int id = pidx < npair ? s_ids[pidx] : -1;
        keys[i] = id < 0 ? inval : (unsigned)id;
        vals[i] = (unsigned short)pidx;
    }
    Sort().sort(keys, vals, s_tmp.sort, 0, bits);
    s_last[threadIdx.x] = keys[kK - 1];
    __syncthreads();   // the sort's storage is free, s_last written
    unsigned prev = threadIdx.x == 0 ? ~0u : s_last[threadIdx.x - 1];
    int nrun = 0;
#pragma unroll
    for (int i = 0; i < kK; ++i) {
        const unsigned pk = i == 0 ? prev : keys[i - 1];
        nrun += (keys[i] != inval && keys[i] != pk) ? 1 : 0;
        if (keys[i] == inval && pk != inval) s_end = threadIdx.x * kK + i;   // one thread: the transition
    }
    int off, total;
    Scan().exclusive_scan(nrun, off, 0, total, s_tmp.scan);
#pragma unroll
    for (int i = 0; i < kK; ++i) {
        const int pos = threadIdx.x * kK + i;
        s_val[pos] = vals[i];
        const unsigned pk = i == 0 ? prev : keys[i - 1];
        if (keys[i] != inval && keys[i] != pk) {
            s_run_id[off] = (int)keys[i];
            s_run_start[off] = (unsigned short)pos;
            ++off;
        }
    }
    __syncthreads();
    const int end = s_end;
    for (int e = threadIdx.x; e < total * kF; e += kTBlock) {
        const int run = e >> 3, d = e & (kF - 1);
        const int a = s_run_start[run], b = run + 1 < total ? s_run_start[run + 1] : end;
        float g = 0.f;
        for (int q = a; q < b; ++q) {
            const int pidx = s_val[q];
            const int lr = pidx / nn_k;
            if (EIK) g = fmaf(fmaf(s_wt[pidx], s_dsdf[lr], s_al[pidx]), gst[lr * kF + d], g);
            else g = fmaf(s_wt[pidx], gst[lr * kF + d], g);
        }
        const int id = s_run_id[run];
        if (fdst) fixed_add(fdst, (int64_t)id * kF + d, g, fscale, fixed_fine_off(st, frows));
        else atomicAdd(grad_features + (int64_t)id * kF + d, g);
    }
    if (!side) return;
    float* const cert = st.cert_fixed ? nullptr : st.certainties;
    unsigned long long* const cfix = (unsigned long long*)st.cert_fixed;
    const double cscale = fixed_scale(st.cert_shift);
    for (int run = threadIdx.x; run < total; run += kTBlock) {
        const int a = s_run_start[run], b = run + 1 < total ? s_run_start[run + 1] : end;
        float wsum = 0.f;
        unsigned long long fsum = 0ull;
        int64_t tmax = -1;
        for (int q = a; q < b; ++q) {
            const int pidx = s_val[q];
            const float w = s_wt[pidx];
            wsum += w;
            if (cfix) fsum += to_fixed(w, cscale);
            const int64_t t = s_rts[pidx / nn_k];
            tmax = t > tmax ? t : tmax;
        }
        const int id = s_run_id[run];
        if (cert) atomicAdd(cert + id, wsum);
        if (cfix) atomicAdd(cfix + id, fsum);
        if (ts_update && tmax >= 0) ts_amax(ts_update, id, tmax);
    }
}

// MF, frozen decoder (no MLP_GRAD), mlp->packed:
//   weighted_first (PIN_TRAIN_DX): x holds s dsdf/dx[0:8] per slot from the forward; the feature
//     terms are dL/dsdf times it, no decoder evaluation here;
//   per-neighbour: each neighbour's input gradient from the matrix-core decoder (mlp_sdf_mfma16)
//     instead of the f32 decoder backward.
// (A per-block LDS pre-sum of the scatter -- hash table on the feature row, 512 tile-sorted slots,
// ~2.7 references per row -- measured slower: 683 vs 467 us, the LDS float atomics alone 470 us.)
// MASK (per-neighbour, PIN_TRAIN_DX): each neighbour's ReLU masks saved by the forward's f32 decode;
//   its input gradient is GEMM2 of the matrix-core decoder alone (mlp_grad8_from_mask) -- no
//   feature re-gather, no hidden layer.
template <bool WF, bool MLP_GRAD, bool MF = false, bool EIK = false, bool MASK = false, bool SORT = false>
__global__ void __launch_bounds__(kTBlock)
k_train_backward(const PinPoints p, const PinMlp m, const float* __restrict__ label, PinTrainCfg c,
                 PinTrainState st, float* __restrict__ grad_features, float* __restrict__ mlp_part,
                 double* __restrict__ loss_part) {
    static_assert(!MF || !MLP_GRAD || (WF && !EIK), "matrix-core backward with a training decoder: weighted_first");
    static_assert(!EIK || !(WF && MF), "analytic eikonal, weighted_first: gx from the forward");
    static_assert(!MASK || (!WF && MF && !MLP_GRAD && !EIK), "mask backward: per-neighbour, frozen decoder");
    constexpr bool kDecode = MF && !WF;               // per-neighbour matrix-core decodes
    constexpr bool kRowDecode = MF && WF && MLP_GRAD; // weighted_first, training decoder: one decode per row
    // weighted_first: one staged gradient row per query row, scattered by the block at the end;
    // per-neighbour: each neighbour's rows are staged and scattered by their own wave inside the
    // neighbour loop (s_nwf: 64 rows x 8 floats + 64 ids per wave, no block barrier), so the block
    // does not hold all k x 8 floats per row (64 KB at k = 8: one wave per SIMD)
    __shared__ float gst[WF ? kTBlock * kF : 1];
    __shared__ float s_nwf[WF ? 1 : kWaves][WF ? 1 : 64 * kF + 64];
    __shared__ float s_mg[MLP_GRAD ? kWaves : 1][MLP_GRAD ? kMgWave : 1];
    __shared__ float s_so[kWaves];
    __shared__ float s_mlp[MF ? 1 : kWSize];
    __shared__ uint4 s_pk[kDecode || kRowDecode ? kPkBytes / 16 : 1];
    __shared__ float s_dsdf[WF && EIK ? kTBlock : 1];
    MlpW mlpw;
    if constexpr (kRowDecode) {   // the decoder scratch is the wave's slice of s_mg (used in turn)
        const uint4* src = (const uint4*)m.packed;
        for (int e = threadIdx.x; e < kPkBytes / 16; e += kTBlock) s_pk[e] = src[e];
        __syncthreads();
        mlpw = MlpW{nullptr, m.sdf_scale, s_mg[threadIdx.x >> 6], (const unsigned char*)s_pk};
    } else {
        mlpw = kDecode ? stage_decoder<true>(m, s_mlp, s_pk)
                       : MF ? MlpW{nullptr, m.sdf_scale, nullptr} : stage_mlp(m, s_mlp);
    }
    const int64_t nrows = c.n_main + 6 * c.n_stencil;
    // the feature terms' destination: grad_features, or this block's replica of it (small batches:
    // the popular points' address lines take 1/replicas of the memory-side atomics each)
    float* const gdst = (grad_features && st.grad_replicas && st.replicas > 1)
                            ? st.grad_replicas + (int64_t)(blockIdx.x % st.replicas) * p.rows * kF
                            : grad_features;
    // the deterministic mode's fixed-point destination (its replica when replicas > 1)
    unsigned long long* const fdst =
        (grad_features && st.grad_fixed)
            ? (unsigned long long*)st.grad_fixed + (st.replicas > 1 ? (int64_t)(blockIdx.x % st.replicas) * p.rows * kF : 0)
            : nullptr;
    const double fscale = fixed_scale(st.fixed_shift);
    const int64_t r = (int64_t)blockIdx.x * kTBlock + threadIdx.x;   // processing slot (per-slot state)
    const bool live = r < nrows;
    // the row it holds (sdf, label)
    const int64_t row = !live ? r : st.sorted_rows ? (int64_t)__float_as_int(((const float4*)st.sorted_rows)[r].w)
                                  : st.order ? st.order[r] : r;
    const int nn_k = c.nn_k;
    const int wave = threadIdx.x >> 6;
    double loss = 0.0;
    const float rs = live ? row_scale(c, row) : 0.f;
    const float dsdf = live ? row_dsdf(c, st.sdf, label, st.row_weight, row, loss) * rs : 0.f;
    loss *= (double)rs;
    if (EIK && live) loss += (double)st.eik_vec[r * (WF ? kEikWf : kEikNwf) + (WF ? 11 : 3)];   // (|g| - 1)^2 term
    const float so = dsdf * mlpw.sdf_scale;           // dL/d(lout output)
    // decoder-parameter products of the block's rows (MLP_GRAD): T, T' accumulators, sum so
    f32x4 accT[4], accE[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) accT[ct] = accE[ct] = (f32x4){0.f, 0.f, 0.f, 0.f};
    float so_sum = 0.f;
    float* mws = MLP_GRAD ? s_mg[wave] : nullptr;
    if (WF && EIK) {
        // feature terms (w_j dsdf + alpha_j) gx[0:8] in the scatter; gx from the forward
        const float* ev = st.eik_vec + (live ? r : 0) * kEikWf;
#pragma unroll
        for (int d = 0; d < kF; ++d) gst[threadIdx.x * kF + d] = live ? ev[12 + d] : 0.f;
        s_dsdf[threadIdx.x] = dsdf;
        if (MLP_GRAD) {
            float x[kD], e[kD], gf[kF];
#pragma unroll
            for (int d = 0; d < kD; ++d) {
                x[d] = live ? st.x[r * kD + d] : 0.f;
                e[d] = live ? ev[d] : 0.f;
            }
#pragma unroll
            for (int d = 0; d < kF; ++d) gf[d] = 0.f;
            const uint64_t mk = decoder_backward_row(mlpw, x, so, gf);   // gf unused: gx came from the forward
            mlp_grad_mfma<true>(mws, mk, so, x, e, accT, accE);
            so_sum += so;
        }
    } else if (kRowDecode) {
        // training decoder on the matrix cores: each row's input gradient and 64 ReLU masks from
        // one decode of the wave's rows, then the decoder-parameter products
        float x[kD], gx[kD];
#pragma unroll
        for (int d = 0; d < kD; ++d) x[d] = live ? st.x[r * kD + d] : 0.f;
        uint64_t mk = 0;
        mlp_sdf_mfma16<true, 0, kD>(mlpw, x, gx, &mk);
#pragma unroll
        for (int d = 0; d < kF; ++d) gst[threadIdx.x * kF + d] = dsdf * gx[d];
        mlp_grad_mfma<false>(mws, mk, so, x, nullptr, accT, accE);
        so_sum += so;
    } else if (WF && MF) {   // PIN_TRAIN_DX: x rows of 8 (s dsdf/dx over the features)
        float4 g0 = make_float4(0.f, 0.f, 0.f, 0.f), g1 = g0;
        if (live) {
            const float4* xr = (const float4*)(st.x + r * kF);
            g0 = xr[0];
            g1 = xr[1];
        }
        const float gv[kF] = {g0.x, g0.y, g0.z, g0.w, g1.x, g1.y, g1.z, g1.w};
#pragma unroll
        for (int d = 0; d < kF; ++d) gst[threadIdx.x * kF + d] = live ? dsdf * gv[d] : 0.f;
    } else if (WF) {
        float x[kD];
#pragma unroll
        for (int d = 0; d < kD; ++d) x[d] = live ? st.x[r * kD + d] : 0.f;
        float gf[kF];
#pragma unroll
        for (int d = 0; d < kF; ++d) gf[d] = 0.f;
        if (MLP_GRAD) {
            const uint64_t mk = decoder_backward_row(mlpw, x, so, gf);
            mlp_grad_mfma<false>(mws, mk, so, x, nullptr, accT, accE);
            so_sum += so;
        } else {
            decoder_backward(mlpw, x, so, gf);
        }
#pragma unroll
        for (int d = 0; d < kF; ++d) gst[threadIdx.x * kF + d] = gf[d];
    } else {
        // per-neighbour decoder backward: dL/dsdf_j = dsdf * w_j (mapper.py:467-468), + alpha_j
        // with the analytic eikonal (whose gx_j[8:] path adds e = [0, w_j R_j^T u])
        float uq[3] = {0.f, 0.f, 0.f};
        if (EIK && live) {
            const float* ev = st.eik_vec + r * kEikNwf;
            uq[0] = ev[0];
            uq[1] = ev[1];
            uq[2] = ev[2];
        }
        for (int j = 0; j < kK; ++j) {
            const int id = (live && j < nn_k) ? st.ids[r * nn_k + j] : -1;
            const bool ok = id >= 0;
            const float w = ok ? st.weights[r * nn_k + j] : 0.f;
            const float al = (EIK && ok) ? st.eik_coef[r * nn_k + j] : 0.f;
            const float coef = dsdf * w + al;        // dL/dsdf_j
            float x[kD];
            if (MASK) {
#pragma unroll
                for (int d = 0; d < kD; ++d) x[d] = 0.f;
            } else if (ok) {
                const float4* fr = (const float4*)(p.features + (int64_t)id * kF);
                const float4 f0 = fr[0], f1 = fr[1];
                const float* v = st.x + (r * nn_k + j) * 3;
                x[0] = f0.x; x[1] = f0.y; x[2] = f0.z; x[3] = f0.w;
                x[4] = f1.x; x[5] = f1.y; x[6] = f1.z; x[7] = f1.w;
                x[8] = v[0]; x[9] = v[1]; x[10] = v[2];
            } else {
#pragma unroll
                for (int d = 0; d < kD; ++d) x[d] = 0.f;
            }
            float gf[kF];
#pragma unroll
            for (int d = 0; d < kF; ++d) gf[d] = 0.f;
            if constexpr (MASK) {
                if (__any(ok)) {   // wave-uniform
                    const uint2 mv = ok ? ((const uint2*)st.x)[r * nn_k + j] : make_uint2(0u, 0u);
                    float g8[kF];
                    mlp_grad8_from_mask(mlpw, ((uint64_t)mv.y << 32) | mv.x, g8);
#pragma unroll
                    for (int d = 0; d < kF; ++d) gf[d] = coef * g8[d];
                }
            } else if constexpr (kDecode) {
                if (__any(ok)) {   // wave-uniform: the whole wave decodes together
                    float g8[kF];
                    mlp_sdf_mfma16<true, 0, kF>(mlpw, x, g8);
#pragma unroll
                    for (int d = 0; d < kF; ++d) gf[d] = coef * g8[d];
                }
            } else if (EIK && MLP_GRAD) {
                float e[kD];
#pragma unroll
                for (int d = 0; d < kF; ++d) e[d] = 0.f;
                float u0 = uq[0], u1 = uq[1], u2 = uq[2];
                if (ok && p.after_pgo) quat_rotate_passive(((const float4*)p.orientations)[id], u0, u1, u2);
                e[kF] = w * u0;
                e[kF + 1] = w * u1;
                e[kF + 2] = w * u2;
                const float soj = coef * mlpw.sdf_scale;
                const uint64_t mk = decoder_backward_row(mlpw, x, soj, gf);
                mlp_grad_mfma<true>(mws, mk, soj, x, e, accT, accE);
                so_sum += soj;
            } else if (MLP_GRAD) {
                const float soj = coef * mlpw.sdf_scale;
                const uint64_t mk = decoder_backward_row(mlpw, x, soj, gf);
                mlp_grad_mfma<false>(mws, mk, soj, x, nullptr, accT, accE);
                so_sum += soj;
            } else if (__any(ok)) {
                decoder_backward(mlpw, x, coef * mlpw.sdf_scale, gf);
            }
            if constexpr (!WF) {
                // this neighbour's 64 gradient rows, scattered by the wave: 8 lanes x 32 contiguous
                // bytes per (row, neighbour), 8 rows per instruction (the shape of the block scatter)
                float* wg = s_nwf[wave];
                int* wid = (int*)(wg + 64 * kF);
                const int lane = threadIdx.x & 63;
                wave_lds_sync();   // the previous neighbour's scatter has read the slots
#pragma unroll
                for (int d = 0; d < kF; ++d) wg[lane * kF + d] = gf[d];
                wid[lane] = ok && gdst ? id : -1;
                wave_lds_sync();
#pragma unroll
                for (int u = 0; u < kF; ++u) {
                    const int e = u * 64 + lane;
                    const int rid = wid[e >> 3];
                    if (rid < 0) continue;
                    if (fdst) fixed_add(fdst, (int64_t)rid * kF + (e & (kF - 1)), wg[e], fscale, fixed_fine_off(st, p.rows));
                    else atomicAdd(gdst + (int64_t)rid * kF + (e & (kF - 1)), wg[e]);
                }
            }
        }
    }
    {
        const double v = [&] {
            double t = loss;
            for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
            return t;
        }();
        if ((threadIdx.x & 63) == 0 && loss_part) loss_part[(int64_t)blockIdx.x * kWaves + wave] = v;
    }
#if defined(PIN_PROF_BWD) && PIN_PROF_BWD >= 3   // profiling variant: decode (and loss) only
    return;
#endif
    if constexpr (MLP_GRAD) mlp_grad_flush<EIK>(s_mg, s_so, accT, accE, so_sum, mlp_part + (int64_t)blockIdx.x * kMlpPart);
    __syncthreads();
    const int64_t row0 = (int64_t)blockIdx.x * kTBlock;
    const int nrow_blk = (int)(nrows - row0 < kTBlock ? nrows - row0 : kTBlock);
    // One LDS buffer for the scatter's staging and, after it, the side-effect table: a buffer the
    // kernel is done with where one fits (the block's scan lists after the per-neighbour
    // matrix-core decodes, the decoder-gradient staging s_mg after mlp_grad_flush), else its own.
    // (A table of its own beside the staging, claimed in the staging pass, measured slower: the
    // larger LDS footprint costs the atomic-bound scatter more occupancy than the reloads it saves.)
    constexpr int kScat = WF ? (EIK ? 3 : 2) * kTBlock * kK : 0;
    constexpr int kNeed = kScat > kSideBufInts ? kScat : kSideBufInts;
    constexpr int kOwn = (MLP_GRAD || kDecode) ? 0 : kNeed;
    static_assert(!kDecode || kNeed <= kTBlock * kListSeg, "scatter staging / side-effect table must fit the scan lists");
    static_assert(!MLP_GRAD || kNeed <= kWaves * kMgWave, "scatter staging must fit the decoder-gradient staging");
    __shared__ int s_own[kOwn > 0 ? kOwn : 1];
    int* const s_pair = MLP_GRAD ? (int*)&s_mg[0][0] : (kDecode ? block_list() : s_own);
#if defined(PIN_PROF_BWD) && PIN_PROF_BWD >= 2   // profiling variant: no feature scatter, no side effects
    return;
#endif
    const bool side = st.certainties || st.cert_fixed || (st.ts_update && st.row_ts);
    bool side_done = false;
    if constexpr (WF) {
        if (grad_features) {
            if constexpr (SORT) {
#if defined(PIN_PROF_BWD) && PIN_PROF_BWD >= 1
                constexpr bool kSide = false;
#else
                constexpr bool kSide = true;
#endif
                feature_scatter_sorted<EIK>(c, st, row0, nrow_blk, gst, s_dsdf, gdst, fdst, fscale, s_pair, p.rows,
                                            side && kSide, row);
                side_done = true;
            } else {
                feature_scatter<EIK>(c, st, row0, nrow_blk, gst, s_dsdf, gdst, fdst, fscale, s_pair, p.rows);
            }
            __syncthreads();   // the staging is read: the table takes the buffer
        }
    }
#if defined(PIN_PROF_BWD) && PIN_PROF_BWD >= 1   // profiling variant: no side effects
    return;
#endif
    if (side && !side_done) train_side_effects(c, st, row0, nrow_blk, row, s_pair);
}

// Per-neighbour (weighted_first False) backward of a frozen decoder, large batches: the feature
// terms pre-summed per feature row over the block's (row, neighbour) pairs before the atomics.
// Each pair's term is dL/dsdf_row * w_j * s dsdf_j/dx[0:8], where dsdf_j/dx comes from neighbour
// j's ReLU mask (saved by the forward) through GEMM2 of the matrix-core decoder.  Instead of
// staging the 2,048 pairs' 32-B terms (64 KB of LDS, one block per CU), the block
//   1. stages only the pairs' ids and weights (coalesced loads, 16 KB),
//   2. radix-sorts the pairs by feature row (rocprim block sort, stable: a run keeps input order),
//   3. evaluates the terms in SORTED order -- 256 pairs per round, each wave's 64 consecutive
//      sorted pairs through one mlp_grad8_from_mask (mask gathered by the pair's index) -- so the
//      pairs of a feature row sit in consecutive lanes: a segmented sum over equal ids (six
//      shuffle steps) leaves each run's total in its last lane, and the runs' totals leave as
//      8 lanes x 32 contiguous bytes per run (the direct scatter's request shape);
//   4. applies the training side effects on the same runs (one certainty add of the run's weight
//      sum, one ts max), as feature_scatter_sorted does.
// A run cut by a wave or round boundary adds its pieces separately (same sum, one more atomic).
// LDS: 8.3 KB decoder image + 16 KB pairs + the sort storage shared with the waves' decoder
// scratch + 4 KB positions -- three blocks per CU.
__global__ void __launch_bounds__(kTBlock)
k_train_backward_nwf_sorted(const PinPoints p, const PinMlp m, const float* __restrict__ label, PinTrainCfg c,
                            PinTrainState st, float* __restrict__ grad_features, double* __restrict__ loss_part) {
    constexpr int kP = kTBlock * kK;
    static_assert(kP <= 65536, "sorted positions are 16-bit");
    using Sort = rocprim::block_radix_sort<unsigned, kTBlock, kK, unsigned short>;
    __shared__ uint4 s_pk[kPkBytes / 16];
    __shared__ union {
        typename Sort::storage_type sort;
        float xs[kWaves][kXsWave];              // mlp_grad8_from_mask's scratch, then the runs' totals
    } s_u;
    __shared__ int s_key[kP];                   // the pairs' ids; after the sort: the id at each position
    __shared__ float s_wt[kP];
    __shared__ unsigned short s_val[kP];        // sorted position -> pair index
    __shared__ float s_dsdf[kTBlock];
    __shared__ int64_t s_rts[kTBlock];
    __shared__ unsigned s_last[kTBlock];
    __shared__ int s_end;
    for (int e = threadIdx.x; e < kPkBytes / 16; e += kTBlock) s_pk[e] = ((const uint4*)m.packed)[e];
    const int nn_k = c.nn_k;
    const int64_t nrows = c.n_main + 6 * c.n_stencil;
    const int64_t row0 = (int64_t)blockIdx.x * kTBlock;
    const int nrow_blk = (int)(nrows - row0 < kTBlock ? nrows - row0 : kTBlock);
    const int npair = nrow_blk * nn_k;
    const int64_t r = row0 + threadIdx.x;
    const bool live = r < nrows;
    const int64_t row = !live ? r : st.sorted_rows ? (int64_t)__float_as_int(((const float4*)st.sorted_rows)[r].w)
                                  : st.order ? st.order[r] : r;
    double loss = 0.0;
    const float rs = live ? row_scale(c, row) : 0.f;
    const float dsdf = live ? row_dsdf(c, st.sdf, label, st.row_weight, row, loss) * rs : 0.f;
    loss *= (double)rs;
    {
        double t = loss;
        for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
        if ((threadIdx.x & 63) == 0 && loss_part) loss_part[(int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6)] = t;
    }
    int64_t* const ts_update = st.row_ts ? st.ts_update : nullptr;
    const bool side = st.certainties || st.cert_fixed || ts_update;
    s_dsdf[threadIdx.x] = dsdf;
    s_rts[threadIdx.x] = (ts_update && live && row < c.n_main) ? st.row_ts[row] : -1;
    for (int e = threadIdx.x; e < npair; e += kTBlock) {
        s_key[e] = st.ids[row0 * nn_k + e];
        s_wt[e] = st.weights[row0 * nn_k + e];
    }
    if (threadIdx.x == 0) s_end = kP;
    __syncthreads();
    // ---- sort the pairs by feature row (as feature_scatter_sorted)
    const int64_t frows = p.rows;
    const unsigned bits = frows >= (int64_t)0x80000000u ? 32u : 32u - (unsigned)__clz((unsigned)frows);
    const unsigned inval = bits >= 32u ? ~0u : (1u << bits) - 1u;
    unsigned keys[kK];
    unsigned short vals[kK];
#pragma unroll
    for (int i = 0; i < kK; ++i) {
        const int pidx = threadIdx.x * kK + i;
        const int id = pidx < npair ? s_key[pidx] : -1;
        keys[i] = id < 0 ? inval : (unsigned)id;
        vals[i] = (unsigned short)pidx;
    }
    Sort().sort(keys, vals, s_u.sort, 0, bits);
    s_last[threadIdx.x] = keys[kK - 1];
    __syncthreads();   // the sort's storage is free, s_last written, every s_key read
    const unsigned prev = threadIdx.x == 0 ? ~0u : s_last[threadIdx.x - 1];
#pragma unroll
    for (int i = 0; i < kK; ++i) {
        const int pos = threadIdx.x * kK + i;
        const unsigned pk = i == 0 ? prev : keys[i - 1];
        if (keys[i] == inval && pk != inval) s_end = pos;   // one thread: the transition
        s_val[pos] = vals[i];
        s_key[pos] = (int)keys[i];
    }
    __syncthreads();   // positions and s_end visible; the sort's storage is free (decoder scratch)
    const int end = s_end;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned long long* const fdst = (grad_features && st.grad_fixed) ? (unsigned long long*)st.grad_fixed : nullptr;
    const double fscale = fixed_scale(st.fixed_shift);
    if (grad_features) {
        const MlpW mw{nullptr, m.sdf_scale, s_u.xs[wave], (const unsigned char*)s_pk};
        const uint2* masks = (const uint2*)st.x + row0 * nn_k;
        const int rounds = (end + kTBlock - 1) / kTBlock;   // block-uniform
        for (int u = 0; u < rounds; ++u) {
            const int pos = u * kTBlock + threadIdx.x;
            const bool ok = pos < end;
            int key = -1;
            float coef = 0.f;
            uint64_t mk = 0;
            if (ok) {
                const int pidx = s_val[pos];
                key = s_key[pos];
                coef = s_dsdf[pidx / nn_k] * s_wt[pidx];
                const uint2 mv = masks[pidx];
                mk = ((uint64_t)mv.y << 32) | mv.x;
            }
            float g[kF];
            if (__any(ok)) {   // wave-uniform: the wave's 64 positions decode together
                float g8[kF];
                mlp_grad8_from_mask(mw, mk, g8);
#pragma unroll
                for (int d = 0; d < kF; ++d) g[d] = coef * g8[d];
                // segmented inclusive sum over lanes of equal id (equal ids are consecutive)
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int ku = __shfl_up(key, o);
                    const bool add = lane >= o && ku == key;
#pragma unroll
                    for (int d = 0; d < kF; ++d) {
                        const float v = __shfl_up(g[d], o);
                        g[d] = add ? g[d] + v : g[d];
                    }
                }
                const int kn = __shfl_down(key, 1);
                const bool tail = ok && (lane == 63 || kn != key);
                // the runs' totals, compacted into the wave's scratch: 8 lanes x 32 B per run
                const uint64_t tails = __ballot(tail);
                const int nt = __popcll(tails);
                float* const ws = s_u.xs[wave];
                int* const wid = (int*)(ws + 64 * kF);
                if (tail) {
                    const int slot = __popcll(tails & ((1ull << lane) - 1ull));
#pragma unroll
                    for (int d = 0; d < kF; ++d) ws[slot * kF + d] = g[d];
                    wid[slot] = key;
                }
                wave_lds_sync();
                for (int e = lane; e < nt * kF; e += 64) {
                    const int rid = wid[e >> 3];
                    if (fdst) fixed_add(fdst, (int64_t)rid * kF + (e & (kF - 1)), ws[e], fscale, fixed_fine_off(st, p.rows));
                    else atomicAdd(grad_features + (int64_t)rid * kF + (e & (kF - 1)), ws[e]);
                }
                wave_lds_sync();   // the next round's decode reuses the scratch
            }
        }
    }
    if (!side) return;
    float* const cert = st.cert_fixed ? nullptr : st.certainties;
    unsigned long long* const cfix = (unsigned long long*)st.cert_fixed;
    const double cscale = fixed_scale(st.cert_shift);
    // one thread per run: the run starts where the sorted id changes
    for (int a = threadIdx.x; a < end; a += kTBlock) {
        const int id = s_key[a];
        if (a > 0 && s_key[a - 1] == id) continue;
        float wsum = 0.f;
        unsigned long long fsum = 0ull;
        int64_t tmax = -1;
        for (int q = a; q < end && s_key[q] == id; ++q) {
            const int pidx = s_val[q];
            const float w = s_wt[pidx];
            wsum += w;
            if (cfix) fsum += to_fixed(w, cscale);
            const int64_t t = s_rts[pidx / nn_k];
            tmax = t > tmax ? t : tmax;
        }
        if (cert) atomicAdd(cert + id, wsum);
        if (cfix) atomicAdd(cfix + id, fsum);
        if (ts_update && tmax >= 0) ts_amax(ts_update, id, tmax);
    }
}
static_assert(kXsWave >= 64 * (kF + 1), "a wave's run totals (8 floats + id per lane) must fit its decoder scratch");

// out[i] += float(sum of the nrep fixed-point accumulators at i * 2^-shift); the accumulators are
// zeroed (pin_fixed_accumulate, and the deterministic pin_train_backward with replica_mode 0)
// parts 2: the feature gradients' coarse and fine parts (fixed_add), the fine part at acc + nrep n
__global__ void __launch_bounds__(kTBlock)
k_fixed_reduce(long long* __restrict__ acc, int nrep, int64_t n, int shift, int parts, float* __restrict__ out) {
    const double inv = 1.0 / fixed_scale(shift);
    long long* const fine = acc + (int64_t)nrep * n;
    for (int64_t e = (int64_t)blockIdx.x * kTBlock + threadIdx.x; e < n; e += (int64_t)gridDim.x * kTBlock) {
        long long s = 0, f = 0;
        for (int k = 0; k < nrep; ++k) {
            s += acc[k * n + e];
            acc[k * n + e] = 0;
            if (parts > 1) {
                f += fine[k * n + e];
                fine[k * n + e] = 0;
            }
        }
        out[e] += parts > 1 ? from_fixed2(s, f, inv) : from_fixed(s, inv);
    }
}

// grad += sum of the replicas, which are zeroed again (pin_train_backward with st.replicas > 1):
// n4 float4 per replica, read once, coalesced
__global__ void __launch_bounds__(kTBlock)
k_replica_reduce(float4* __restrict__ rep, int nrep, int64_t n4, float4* __restrict__ grad) {
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t e = (int64_t)blockIdx.x * kTBlock + threadIdx.x; e < n4; e += (int64_t)gridDim.x * kTBlock) {
        float4 a = z;
        for (int k = 0; k < nrep; ++k) {
            const float4 v = rep[k * n4 + e];
            rep[k * n4 + e] = z;
            a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
        }
        float4 g = grad[e];
        g.x += a.x; g.y += a.y; g.z += a.z; g.w += a.w;
        grad[e] = g;
    }
}

__global__ void __launch_bounds__(1024) k_loss_final(const double* __restrict__ part, int64_t n,
                                                     double* __restrict__ out) {
    __shared__ double red[16];
    double v = 0.0;
#pragma unroll 8   // the loads in flight together (the adds keep their order)
    for (int64_t i = threadIdx.x; i < n; i += 1024) v += part[i];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int w = 0; w < 16; ++w) t += red[w];
        out[0] = t;
    }
}

// Decoder-parameter gradients from the blocks' partials (fixed order): block b reduces hidden
// units 4b..4b+3 (64 products of T, and of T' with the analytic eikonal), 4 waves over interleaved
// block ranges, then mlp_grad += dW1 = w2 o (T + s T')[:, 0:11], db1 = w2 o T[:, 11],
// dW2 = rowwise W1 . (T + s T')[:, 0:11] + b1 o T[:, 11]; block 0 also adds db2 = sum so.
// Block kH / 4 (launched when loss_out is wanted) reduces the loss partials instead, so that a
// training-decoder backward ends with one launch, not k_loss_final + this.
__global__ void __launch_bounds__(kTBlock) k_mlp_grad_final(const float* __restrict__ part, int64_t nblk, int extra,
                                                           PinMlp m, float* __restrict__ out,
                                                           const double* __restrict__ lpart, int64_t nl,
                                                           double* __restrict__ loss_out) {
    __shared__ float red[kWaves][2][64];
    __shared__ float s_b2[kWaves];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (blockIdx.x == kH / 4) {   // the loss: fixed-order sum of the per-wave partials
        __shared__ double lred[kWaves];
        double v = 0.0;
        for (int64_t k = threadIdx.x; k < nl; k += kTBlock) v += lpart[k];
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0) lred[wave] = v;
        __syncthreads();
        if (threadIdx.x == 0) {
            double tot = 0.0;
            for (int w = 0; w < kWaves; ++w) tot += lred[w];
            loss_out[0] = tot;
        }
        return;
    }
    const int c = 4 * blockIdx.x + (lane >> 4), i = lane & 15;
    const int e = c * 16 + i;
    float t = 0.f, te = 0.f, b2 = 0.f;
#pragma unroll 8
    for (int64_t b = wave; b < nblk; b += kWaves) {
        const float* pb = part + b * kMlpPart;
        t += pb[e];
        if (extra) te += pb[kTSize + e];
    }
    if (blockIdx.x == 0) {
        for (int64_t b = threadIdx.x; b < nblk; b += kTBlock) b2 += part[b * kMlpPart + 2 * kTSize];
        b2 = wave_sum_f(b2);
        if (lane == 0) s_b2[wave] = b2;
    }
    red[wave][0][lane] = t;
    red[wave][1][lane] = te;
    __syncthreads();
    if (wave != 0) return;
    t = 0.f;
    te = 0.f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
        t += red[w][0][lane];
        te += red[w][1][lane];
    }
    const float w2 = m.W2[c];
    const float v = fmaf(m.sdf_scale, te, t);
    float d2 = 0.f;
    if (i < kD) {
        out[c * kD + i] += w2 * v;
        d2 = m.W1[c * kD + i] * v;
    } else if (i == kD) {
        out[kH * kD + c] += w2 * t;
        d2 = m.b1[c] * t;
    }
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) d2 += __shfl_xor(d2, off);   // the 16 lanes of hidden unit c
    if (i == 0) out[kH * kD + kH + c] += d2;
    if (blockIdx.x == 0 && lane == 0) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) s += s_b2[w];
        out[kMlpGrad - 1] += s;
    }
}

// ----------------------------------------------------------------------------- Decoder.sdf rows
// The drop-in Decoder.sdf (model/decoder.py:66-88) on rows x [n, 11] and its autograd: the
// forward, the first-order backward (input gradient, parameter products) and the double backward
// of the input gradient (the analytic eikonal through get_gradient(create_graph=True),
// utils/tools.py:174-184).  The ReLU masks are piecewise constant, so the second-order terms are
// bilinear in (go, e): with u_c = W1[c] . e,
//   d(gx . e)/d go = s sum_c w2_c m_c u_c,  d/dW1[c][i] = s w2_c sum_r m_c go e_i,
//   d/dw2_c = s W1[c] . sum_r m_c go e     -- k_mlp_grad_final's T' terms with e' = go e.
constexpr int kMlpRowBlocks = 512;    // persistent grid of the row backward: bounded partials (k_mlp_grad_final reads them all)

__global__ void __launch_bounds__(kTBlock)
k_mlp_forward(PinMlp m, const float* __restrict__ x, int64_t n, float* __restrict__ out) {
    __shared__ float s_w[kWSize];
    const MlpW mw = stage_mlp(m, s_w);
    for (int64_t r = (int64_t)blockIdx.x * kTBlock + threadIdx.x; r < n; r += (int64_t)gridDim.x * kTBlock) {
        float xv[kD];
#pragma unroll
        for (int i = 0; i < kD; ++i) xv[i] = x[r * kD + i];
        float g1[1];
        out[r] = mlp_sdf<false, 0, 1>(mw, xv, g1);
    }
}

// GX: gx[r] = go_r s W1^T (w2 o m);  DGO: d_go[r] = s sum_c w2_c m_c (W1[c] . e_r);
// FIRST / SECOND: the block's parameter products (T from so = go s, T' from go e) into part
template <bool GX, bool DGO, bool FIRST, bool SECOND>
__global__ void __launch_bounds__(kTBlock)
k_mlp_backward(PinMlp m, const float* __restrict__ x, int64_t n, const float* __restrict__ go,
               const float* __restrict__ e, float* __restrict__ gx, float* __restrict__ d_go,
               float* __restrict__ part) {
    constexpr bool PARAMS = FIRST || SECOND;
    __shared__ float s_w[kWSize];
    __shared__ float s_mg[PARAMS ? kWaves : 1][PARAMS ? kMgWave : 1];
    __shared__ float s_so[kWaves];
    const MlpW mw = stage_mlp(m, s_w);
    const float s = m.sdf_scale;
    f32x4 accT[4], accE[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) accT[k] = accE[k] = (f32x4){0.f, 0.f, 0.f, 0.f};
    float so_sum = 0.f;
    const int64_t stride = (int64_t)gridDim.x * kTBlock;
    const int64_t iters = (n + stride - 1) / stride;   // uniform over the block: every lane joins the MFMAs
    for (int64_t it = 0; it < iters; ++it) {
        const int64_t r = it * stride + (int64_t)blockIdx.x * kTBlock + threadIdx.x;
        const bool live = r < n;
        float xv[kD], ev[kD];
        float g = 0.f;
#pragma unroll
        for (int i = 0; i < kD; ++i) {
            xv[i] = live ? x[r * kD + i] : 0.f;
            ev[i] = (live && (DGO || SECOND)) ? e[r * kD + i] : 0.f;
        }
        if (live && (GX || PARAMS)) g = go[r];
        float ga[kD];
#pragma unroll
        for (int i = 0; i < kD; ++i) ga[i] = 0.f;
        float dg = 0.f;
        uint32_t lo = 0u, hi = 0u;
#pragma unroll 2
        for (int c = 0; c < kH; ++c) {
            float wr[kWRow];
            load_row(mw.w, c, wr);
            float acc = 0.f;
#pragma unroll
            for (int i = 0; i < kD; ++i) acc = fmaf(wr[i], xv[i], acc);
            const bool on = acc + mw.w[kWB1 + c] > 0.f;
            const float a = on ? mw.w[kWW2 + c] : 0.f;
            if (GX) {
#pragma unroll
                for (int i = 0; i < kD; ++i) ga[i] = fmaf(a, wr[i], ga[i]);
            }
            if (DGO) {
                float u = 0.f;
#pragma unroll
                for (int i = 0; i < kD; ++i) u = fmaf(wr[i], ev[i], u);
                dg = fmaf(a, u, dg);
            }
            const uint32_t bit = on ? 1u << (c & 31) : 0u;
            if (c < 32) lo |= bit; else hi |= bit;
        }
        if (live && GX) {
            const float k = s * g;
#pragma unroll
            for (int i = 0; i < kD; ++i) gx[r * kD + i] = ga[i] * k;
        }
        if (live && DGO) d_go[r] = dg * s;
        if constexpr (PARAMS) {
            const uint64_t mask = live ? (((uint64_t)hi << 32) | lo) : 0ull;
            const float so = (FIRST && live) ? g * s : 0.f;
            float e2[kD];
#pragma unroll
            for (int i = 0; i < kD; ++i) e2[i] = SECOND ? g * ev[i] : 0.f;
            mlp_grad_mfma<SECOND>(s_mg[threadIdx.x >> 6], mask, so, xv, e2, accT, accE);
            so_sum += so;
        }
    }
    if constexpr (PARAMS) mlp_grad_flush<SECOND>(s_mg, s_so, accT, accE, so_sum, part + (int64_t)blockIdx.x * kMlpPart);
}

// torch.optim.Adam (single-tensor form, weight_decay 0), four elements per thread:
//   m = m + (1-b1)(g - m);  v = v b2 + ((1-b1') g) g;  p += (-lr/bc1 * m) / (sqrt(v)/sqrt(bc2) + eps)
// Element i's gradient sits at (i/8)*grad_stride + i%8 (64-B accumulator rows: lanes 0..7).
__device__ __forceinline__ float adam_one(float& p, float g, float& m, float& v, const PinAdamStep& a) {
    m = m + a.one_minus_beta1 * (g - m);
    v = v * a.beta2;
    v = v + (a.one_minus_beta2 * g) * g;
    const float denom = sqrtf(v) / a.bias_correction2_sqrt + a.eps;
    p = p + (a.neg_step_size * m) / denom;
    return p;
}

// dense Adam over 4 consecutive floats per thread (k_adam, k_adam_step_segments)
__device__ __forceinline__ void adam_dense_body(int64_t t, float* __restrict__ prm, float* __restrict__ grad,
                                                float* __restrict__ m_, float* __restrict__ v_, int64_t n,
                                                const PinAdamStep& a) {
    const int64_t i0 = 4 * t;
    if (i0 >= n) return;
    if (i0 + 4 <= n) {
        const int64_t gi = a.grad_stride == 8 ? i0 : (i0 >> 3) * a.grad_stride + (i0 & 7);
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        float4 p = *(float4*)(prm + i0), g = *(float4*)(grad + gi);
        float4 m = (a.zero_grad & 2) ? z : *(float4*)(m_ + i0), v = (a.zero_grad & 2) ? z : *(float4*)(v_ + i0);
        adam_one(p.x, g.x, m.x, v.x, a);
        adam_one(p.y, g.y, m.y, v.y, a);
        adam_one(p.z, g.z, m.z, v.z, a);
        adam_one(p.w, g.w, m.w, v.w, a);
        *(float4*)(prm + i0) = p;
        *(float4*)(m_ + i0) = m;
        *(float4*)(v_ + i0) = v;
        if (a.zero_grad & 1) *(float4*)(grad + gi) = make_float4(0.f, 0.f, 0.f, 0.f);
        return;
    }
    for (int64_t i = i0; i < n; ++i) {   // tail (contiguous layout only: strided needs n % 8 == 0)
        float p = prm[i], m = (a.zero_grad & 2) ? 0.f : m_[i], v = (a.zero_grad & 2) ? 0.f : v_[i];
        adam_one(p, grad[i], m, v, a);
        prm[i] = p;
        m_[i] = m;
        v_[i] = v;
        if (a.zero_grad & 1) grad[i] = 0.f;
    }
}

__global__ void __launch_bounds__(kTBlock)
k_adam(float* __restrict__ prm, float* __restrict__ grad, float* __restrict__ m_, float* __restrict__ v_, int64_t n,
       PinAdamStep a) {
    adam_dense_body((int64_t)blockIdx.x * kTBlock + threadIdx.x, prm, grad, m_, v_, n, a);
}

// Adam on listed rows of a [rows, 8] parameter (the owned rows of a spatially sharded mapper):
// one thread per (row, half row), the same arithmetic as k_adam; the rows' gradients are zeroed
__global__ void __launch_bounds__(kTBlock)
k_adam_rows(float* __restrict__ prm, float* __restrict__ grad, float* __restrict__ m_, float* __restrict__ v_,
            const int64_t* __restrict__ rows, int64_t nrows, PinAdamStep a) {
    const int64_t t = (int64_t)blockIdx.x * kTBlock + threadIdx.x;
    if (t >= 2 * nrows) return;
    const int64_t i0 = rows[t >> 1] * kF + 4 * (t & 1);
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    float4 p = *(float4*)(prm + i0), g = *(float4*)(grad + i0);
    float4 m = (a.zero_grad & 2) ? z : *(float4*)(m_ + i0), v = (a.zero_grad & 2) ? z : *(float4*)(v_ + i0);
    adam_one(p.x, g.x, m.x, v.x, a);
    adam_one(p.y, g.y, m.y, v.y, a);
    adam_one(p.z, g.z, m.z, v.z, a);
    adam_one(p.w, g.w, m.w, v.w, a);
    *(float4*)(prm + i0) = p;
    *(float4*)(m_ + i0) = m;
    *(float4*)(v_ + i0) = v;
    if (a.zero_grad & 1) *(float4*)(grad + i0) = make_float4(0.f, 0.f, 0.f, 0.f);
}

// Adam over up to kMaxSeg separate parameter tensors whose gradients / moments lie end to end in
// contiguous grad / m / v (the decoder's W1, b1, W2, b2 after one backward): one launch for all.
constexpr int kMaxSeg = 8;
struct AdamSegs {
    float* p[kMaxSeg];
    int64_t off[kMaxSeg + 1];
    int n;
};

// one element of the segments (k_adam_segments, k_adam_step_segments)
__device__ __forceinline__ void adam_segment_body(int64_t t, const AdamSegs& sg, float* __restrict__ grad,
                                                  float* __restrict__ m_, float* __restrict__ v_,
                                                  const PinAdamStep& a, float* copy = nullptr) {
    if (t >= sg.off[sg.n]) return;
    int s = 0;
#pragma unroll
    for (int k = 1; k < kMaxSeg; ++k) s += (k < sg.n && t >= sg.off[k]) ? 1 : 0;
    float* prm = sg.p[s] + (t - sg.off[s]);
    float p = *prm, m = (a.zero_grad & 2) ? 0.f : m_[t], v = (a.zero_grad & 2) ? 0.f : v_[t];
    adam_one(p, grad[t], m, v, a);
    *prm = p;
    if (copy) copy[t] = p;   // the stepped value, also into a block-local copy (k_adam_train)
    m_[t] = m;
    v_[t] = v;
    if (a.zero_grad & 1) grad[t] = 0.f;
}

__global__ void __launch_bounds__(kTBlock)
k_adam_segments(AdamSegs sg, float* __restrict__ grad, float* __restrict__ m_, float* __restrict__ v_, PinAdamStep a) {
    adam_segment_body((int64_t)blockIdx.x * kTBlock + threadIdx.x, sg, grad, m_, v_, a);
}

// The feature Adam and the decoder's segments in one launch (a training mapper iteration): the
// first nb_dense blocks run k_adam's body, the rest k_adam_segments' (the same scalars).
__global__ void __launch_bounds__(kTBlock)
k_adam_step_segments(float* __restrict__ prm, float* __restrict__ grad, float* __restrict__ m_,
                     float* __restrict__ v_, int64_t n, int64_t nb_dense, AdamSegs sg, float* __restrict__ sgrad,
                     float* __restrict__ sm, float* __restrict__ sv, PinAdamStep a) {
    if ((int64_t)blockIdx.x < nb_dense) adam_dense_body((int64_t)blockIdx.x * kTBlock + threadIdx.x, prm, grad, m_, v_, n, a);
    else adam_segment_body(((int64_t)blockIdx.x - nb_dense) * kTBlock + threadIdx.x, sg, sgrad, sm, sv, a);
}

// One training iteration's optimiser step (pin_adam_step_train): with decoder segments, block 0
// steps them and then, with out set, writes the decoder's matrix-core image from the stepped
// parameters (mlp_pack_block); the other nb_dense blocks step the features four floats per thread,
// their gradient plus the sum of the backward's replicas (zeroed again).
__global__ void __launch_bounds__(kTBlock)
k_adam_train(float* __restrict__ prm, float* __restrict__ grad, float* __restrict__ m_, float* __restrict__ v_,
             int64_t n, int64_t nb_dense, float* __restrict__ rep, int nrep, long long* __restrict__ fix, int nfix,
             int fshift, AdamSegs sg, float* __restrict__ sgrad, float* __restrict__ sm, float* __restrict__ sv,
             PinMlp mlp, unsigned char* __restrict__ out, PinAdamStep a) {
    // the decoder's block first (dispatched first: the pack after its step is the longest chain)
    const int64_t bid = (int64_t)blockIdx.x - (sg.n > 0 ? 1 : 0);
    if (bid >= 0) {
        const int64_t i0 = 4 * (bid * kTBlock + threadIdx.x);
        if (fix && i0 < n) {   // deterministic mode: grad + float(integer sums of the fixed-point replicas)
            long long s[4] = {0, 0, 0, 0}, f[4] = {0, 0, 0, 0};
            for (int k = 0; k < nfix; ++k) {
                longlong2* r = (longlong2*)(fix + k * n + i0);
                longlong2* q = (longlong2*)(fix + (nfix + k) * n + i0);   // the fine part (fixed_add)
                const longlong2 v0 = r[0], v1 = r[1], w0 = q[0], w1 = q[1];
                r[0] = r[1] = make_longlong2(0, 0);
                q[0] = q[1] = make_longlong2(0, 0);
                s[0] += v0.x; s[1] += v0.y; s[2] += v1.x; s[3] += v1.y;
                f[0] += w0.x; f[1] += w0.y; f[2] += w1.x; f[3] += w1.y;
            }
            const double inv = 1.0 / fixed_scale(fshift);
            float4 g = *(float4*)(grad + i0);
            g.x += from_fixed2(s[0], f[0], inv); g.y += from_fixed2(s[1], f[1], inv);
            g.z += from_fixed2(s[2], f[2], inv); g.w += from_fixed2(s[3], f[3], inv);
            *(float4*)(grad + i0) = g;
        } else if (nrep > 1 && i0 < n) {   // n % 4 == 0 (checked by the host)
            float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int k = 0; k < nrep; ++k) {
                float4* r = (float4*)(rep + k * n + i0);
                const float4 v = *r;
                *r = make_float4(0.f, 0.f, 0.f, 0.f);
                s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
            }
            float4 g = *(float4*)(grad + i0);   // the order of k_replica_reduce: grad + (sum of replicas)
            g.x += s.x; g.y += s.y; g.z += s.z; g.w += s.w;
            *(float4*)(grad + i0) = g;
        }
        adam_dense_body(bid * kTBlock + threadIdx.x, prm, grad, m_, v_, n, a);
        return;
    }
    // with the decoder's layout (W1 | b1 | W2 | b2 end to end, checked by the host) the stepped
    // values also go to LDS, and the pack reads them there (no global round trip behind a fence)
    __shared__ float s_dec[kMlpGrad];
    // the segments ARE mlp's W1 | b1 | W2 | b2, in that order (sizes alone would not tell b1 from W2)
    const bool lds = out && sg.n == 4 && sg.off[4] == kMlpGrad && sg.off[1] == kH * kD && sg.off[2] == kH * kD + kH &&
                     sg.off[3] == kH * kD + 2 * kH && sg.p[0] == mlp.W1 && sg.p[1] == mlp.b1 && sg.p[2] == mlp.W2 &&
                     sg.p[3] == mlp.b2;
    if (lds) {
        // the decoder's kMlpGrad elements in up to four per thread: every load issued before the
        // first step (one memory latency on the chain to the pack instead of four in turn)
        static_assert(kMlpGrad <= 4 * kTBlock, "decoder step: four elements per thread");
        float p[4], g[4], m[4], v[4];
        float* at[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int t = threadIdx.x + i * kTBlock;
            if (t < kMlpGrad) {
                const int sgi = (t >= sg.off[1] ? 1 : 0) + (t >= sg.off[2] ? 1 : 0) + (t >= sg.off[3] ? 1 : 0);
                at[i] = sg.p[sgi] + (t - sg.off[sgi]);
                p[i] = *at[i];
                g[i] = sgrad[t];
                m[i] = (a.zero_grad & 2) ? 0.f : sm[t];
                v[i] = (a.zero_grad & 2) ? 0.f : sv[t];
            }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int t = threadIdx.x + i * kTBlock;
            if (t < kMlpGrad) {
                adam_one(p[i], g[i], m[i], v[i], a);
                *at[i] = p[i];
                s_dec[t] = p[i];
                sm[t] = m[i];
                sv[t] = v[i];
                if (a.zero_grad & 1) sgrad[t] = 0.f;
            }
        }
    } else {
        for (int64_t t = threadIdx.x; t < sg.off[sg.n]; t += kTBlock) adam_segment_body(t, sg, sgrad, sm, sv, a);
    }
    if (out) {
        if (lds) {
            __syncthreads();
            PinMlp ml = mlp;
            ml.W1 = s_dec;
            ml.b1 = s_dec + kH * kD;
            ml.W2 = s_dec + kH * kD + kH;
            ml.b2 = s_dec + kH * kD + 2 * kH;
            mlp_pack_block(ml, out);
        } else {
            __threadfence();   // the stepped parameters, read back by the pack below (other threads' writes)
            __syncthreads();
            mlp_pack_block(mlp, out);
        }
    }
}

}  // namespace

extern "C" {

int pin_mlp_forward(const PinMlp* mlp, const float* x, int64_t n, float* out, void* stream) {
    if (!mlp || !mlp->W1 || !mlp->b1 || !mlp->W2 || !mlp->b2 || n < 0 || (n > 0 && (!x || !out))) return PIN_ERR_ARG;
    if (n == 0) return PIN_OK;
    const int64_t nb = std::min<int64_t>((n + kTBlock - 1) / kTBlock, 8192);
    hipLaunchKernelGGL(k_mlp_forward, dim3((unsigned)nb), dim3(kTBlock), 0, as_stream(stream), *mlp, x, n, out);
    return launch_status();
}

int64_t pin_mlp_backward_workspace_bytes(int64_t n) {
    const int64_t nb = std::max<int64_t>(1, std::min<int64_t>((n + kTBlock - 1) / kTBlock, kMlpRowBlocks));
    return nb * kMlpPart * (int64_t)sizeof(float);
}

int pin_mlp_backward(const PinMlp* mlp, const float* x, int64_t n, const float* go, const float* e, int32_t flags,
                     float* gx, float* d_go, float* mlp_grad, void* workspace, void* stream) {
    const bool first = (flags & PIN_MLP_GRAD_FIRST) != 0, second = (flags & PIN_MLP_GRAD_SECOND) != 0;
    const bool params = first || second;
    if (!mlp || !mlp->W1 || !mlp->b1 || !mlp->W2 || !mlp->b2 || n < 0) return PIN_ERR_ARG;
    if ((flags & ~(PIN_MLP_GRAD_FIRST | PIN_MLP_GRAD_SECOND)) != 0) return PIN_ERR_ARG;
    if (params && (!mlp_grad || !workspace)) return PIN_ERR_ARG;
    if (n > 0 && (!x || ((gx || params) && !go) || ((d_go || second) && !e))) return PIN_ERR_ARG;
    if (n == 0) return PIN_OK;
    auto st = as_stream(stream);
    const int64_t nb = std::max<int64_t>(1, std::min<int64_t>((n + kTBlock - 1) / kTBlock, kMlpRowBlocks));
    float* part = (float*)workspace;
    const int key = (gx ? 1 : 0) | (d_go ? 2 : 0) | (first ? 4 : 0) | (second ? 8 : 0);
#define PIN_MLP_BWD(K)                                                                                           \
    case K:                                                                                                      \
        hipLaunchKernelGGL((k_mlp_backward<(K & 1) != 0, (K & 2) != 0, (K & 4) != 0, (K & 8) != 0>), dim3((unsigned)nb), \
                           dim3(kTBlock), 0, st, *mlp, x, n, go, e, gx, d_go, part);                             \
        break;
    switch (key) {
        case 0: return PIN_OK;
        PIN_MLP_BWD(1) PIN_MLP_BWD(2) PIN_MLP_BWD(3) PIN_MLP_BWD(4) PIN_MLP_BWD(5) PIN_MLP_BWD(6) PIN_MLP_BWD(7)
        PIN_MLP_BWD(8) PIN_MLP_BWD(9) PIN_MLP_BWD(10) PIN_MLP_BWD(11) PIN_MLP_BWD(12) PIN_MLP_BWD(13)
        PIN_MLP_BWD(14) PIN_MLP_BWD(15)
    }
#undef PIN_MLP_BWD
    if (params)
        hipLaunchKernelGGL(k_mlp_grad_final, dim3(kH / 4), dim3(kTBlock), 0, st, part, nb, second ? 1 : 0, *mlp,
                           mlp_grad, (const double*)nullptr, (int64_t)0, (double*)nullptr);
    return launch_status();
}


static int adam_segs(float* const* params, const int64_t* sizes, int nseg, AdamSegs& sg) {
    if (!params || !sizes || nseg < 1 || nseg > kMaxSeg) return PIN_ERR_ARG;
    sg = AdamSegs{};
    sg.n = nseg;
    sg.off[0] = 0;
    for (int k = 0; k < nseg; ++k) {
        if (sizes[k] < 0 || (sizes[k] > 0 && !params[k])) return PIN_ERR_ARG;
        sg.p[k] = params[k];
        sg.off[k + 1] = sg.off[k] + sizes[k];
    }
    return PIN_OK;
}

int pin_adam_step_segments(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                           float* const* params, const int64_t* sizes, int nseg, float* seg_grad, float* seg_exp_avg,
                           float* seg_exp_avg_sq, const PinAdamStep* a, void* stream) {
    if (!a || n < 0 || (n > 0 && (!param || !grad || !exp_avg || !exp_avg_sq)) || !seg_grad || !seg_exp_avg ||
        !seg_exp_avg_sq)
        return PIN_ERR_ARG;
    if (a->grad_stride != 8) return PIN_ERR_UNSUPPORTED;
    AdamSegs sg;
    const int rc = adam_segs(params, sizes, nseg, sg);
    if (rc != PIN_OK) return rc;
    const int64_t nb_dense = (n + 4 * kTBlock - 1) / (4 * kTBlock);
    const int64_t nb_seg = (sg.off[nseg] + kTBlock - 1) / kTBlock;
    if (nb_dense + nb_seg == 0) return PIN_OK;
    hipLaunchKernelGGL(k_adam_step_segments, dim3((unsigned)(nb_dense + nb_seg)), dim3(kTBlock), 0, as_stream(stream),
                       param, grad, exp_avg, exp_avg_sq, n, nb_dense, sg, seg_grad, seg_exp_avg, seg_exp_avg_sq, *a);
    return launch_status();
}

int pin_adam_step_train(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                        float* grad_replicas, int32_t replicas, int64_t* grad_fixed, int32_t fixed_shift,
                        float* const* params, const int64_t* sizes, int nseg, float* seg_grad, float* seg_exp_avg,
                        float* seg_exp_avg_sq, const PinMlp* mlp, void* packed, const PinAdamStep* a, void* stream) {
    if (!a || n < 0 || (n > 0 && (!param || !grad || !exp_avg || !exp_avg_sq))) return PIN_ERR_ARG;
    if (a->grad_stride != 8) return PIN_ERR_UNSUPPORTED;
    const bool rep = grad_replicas && replicas > 1;
    if (rep && (n % 4 || ((uintptr_t)grad_replicas & 15))) return PIN_ERR_ARG;
    if (grad_fixed && (grad_replicas || n % 4 || ((uintptr_t)grad_fixed & 15) || fixed_shift < 0 || fixed_shift > 62))
        return PIN_ERR_ARG;
    AdamSegs sg{};
    sg.n = 0;
    if (nseg > 0) {
        if (!seg_grad || !seg_exp_avg || !seg_exp_avg_sq) return PIN_ERR_ARG;
        const int rc = adam_segs(params, sizes, nseg, sg);
        if (rc != PIN_OK) return rc;
    } else if (nseg < 0) {
        return PIN_ERR_ARG;
    }
    const bool pack = nseg > 0 && mlp && packed;
    if (pack && (!mlp->W1 || !mlp->b1 || !mlp->W2 || !mlp->b2 || ((uintptr_t)packed & 15))) return PIN_ERR_ARG;
    PinMlp m{};
    if (pack) m = *mlp;
    const int64_t nb_dense = (n + 4 * kTBlock - 1) / (4 * kTBlock);
    const int64_t nb = nb_dense + (nseg > 0 ? 1 : 0);
    if (nb == 0) return PIN_OK;
    hipLaunchKernelGGL(k_adam_train, dim3((unsigned)nb), dim3(kTBlock), 0, as_stream(stream), param, grad, exp_avg,
                       exp_avg_sq, n, nb_dense, rep ? grad_replicas : nullptr, rep ? (int)replicas : 0,
                       (long long*)grad_fixed, replicas > 1 ? (int)replicas : 1, (int)fixed_shift, sg, seg_grad,
                       seg_exp_avg, seg_exp_avg_sq, m, pack ? (unsigned char*)packed : nullptr, *a);
    return launch_status();
}

int pin_fixed_accumulate(int64_t* acc, int32_t nrep, int64_t n, int32_t shift, int32_t parts, float* out,
                         void* stream) {
    if (n < 0 || (n > 0 && (!acc || !out)) || shift < 0 || shift > 62 || parts < 1 || parts > 2) return PIN_ERR_ARG;
    if (n == 0) return PIN_OK;
    const int64_t nb = (n + kTBlock - 1) / kTBlock;
    hipLaunchKernelGGL(k_fixed_reduce, dim3((unsigned)(nb < 2048 ? nb : 2048)), dim3(kTBlock), 0, as_stream(stream),
                       (long long*)acc, nrep > 1 ? (int)nrep : 1, n, (int)shift, (int)parts, out);
    return launch_status();
}

int pin_adam_segments(float* const* params, const int64_t* sizes, int nseg, float* grad, float* exp_avg,
                      float* exp_avg_sq, const PinAdamStep* a, void* stream) {
    if (!a || !grad || !exp_avg || !exp_avg_sq) return PIN_ERR_ARG;
    if (a->grad_stride != 8) return PIN_ERR_UNSUPPORTED;
    AdamSegs sg;
    const int rc = adam_segs(params, sizes, nseg, sg);
    if (rc != PIN_OK) return rc;
    if (sg.off[nseg] == 0) return PIN_OK;
    hipLaunchKernelGGL(k_adam_segments, grid_for(sg.off[nseg]), dim3(kTBlock), 0, as_stream(stream), sg, grad, exp_avg,
                       exp_avg_sq, *a);
    return launch_status();
}

int pin_adam_rows(float* param, float* grad, float* exp_avg, float* exp_avg_sq, const int64_t* rows, int64_t nrows,
                  const PinAdamStep* a, void* stream) {
    if (!a || nrows < 0 || (nrows > 0 && (!param || !grad || !exp_avg || !exp_avg_sq || !rows))) return PIN_ERR_ARG;
    if (a->grad_stride != 8) return PIN_ERR_UNSUPPORTED;
    if (nrows == 0) return PIN_OK;
    if (((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) & 15) return PIN_ERR_ARG;
    hipLaunchKernelGGL(k_adam_rows, grid_for(2 * nrows), dim3(kTBlock), 0, as_stream(stream), param, grad, exp_avg,
                       exp_avg_sq, rows, nrows, *a);
    return launch_status();
}

int pin_train_rows(const float* coord, const PinTrainCfg* cfg, float* rows_out, void* stream) {
    if (!cfg || cfg->n_main < 0 || cfg->n_stencil < 0 || cfg->decimation < 1) return PIN_ERR_ARG;
    const int64_t rows = cfg->n_main + 6 * cfg->n_stencil;
    if (rows == 0) return PIN_OK;
    if (!coord || !rows_out) return PIN_ERR_ARG;
    hipLaunchKernelGGL(k_train_rows, grid_for(rows), dim3(kTBlock), 0, as_stream(stream), coord, *cfg, rows_out);
    return launch_status();
}

int pin_pool_pack(const float* coord, const float* label, const int64_t* ts, const float* weight, int64_t n,
                  float* packed, void* stream) {
    if (n < 0 || (n > 0 && (!coord || !label || !packed)) || ((uintptr_t)packed & 15)) return PIN_ERR_ARG;
    if (n == 0) return PIN_OK;
    hipLaunchKernelGGL(k_pool_pack, grid_for(n), dim3(kTBlock), 0, as_stream(stream), coord, label, ts, weight, n,
                       (float4*)packed);
    return launch_status();
}

static int gather_packed_args(const float* packed_pool, int64_t pool_rows, const PinTrainCfg* cfg,
                              const float* rows_out, const float* label_out) {
    if (!cfg || cfg->n_main < 0 || cfg->n_stencil < 0 || cfg->decimation < 1) return PIN_ERR_ARG;
    if (cfg->n_stencil > 0 && (cfg->n_stencil - 1) * (int64_t)cfg->decimation >= cfg->n_main) return PIN_ERR_ARG;
    if (cfg->n_main == 0) return PIN_OK;
    if (!packed_pool || ((uintptr_t)packed_pool & 15) || !rows_out || !label_out || pool_rows < 1) return PIN_ERR_ARG;
    return PIN_OK;
}

int pin_train_gather_packed(const float* packed_pool, int64_t pool_rows, const int64_t* index, const PinTrainCfg* cfg,
                            float* rows_out, float* label_out, int64_t* ts_out, float* weight_out, int32_t* error,
                            void* stream) {
    const int rc = gather_packed_args(packed_pool, pool_rows, cfg, rows_out, label_out);
    if (rc != PIN_OK || cfg->n_main == 0) return rc;
    if (!index) return PIN_ERR_ARG;
    hipLaunchKernelGGL(k_train_gather_packed, grid_for(cfg->n_main), dim3(kTBlock), 0, as_stream(stream),
                       (const float4*)packed_pool, pool_rows, index, cfg->n_main, nullptr, (int64_t)0, nullptr, *cfg,
                       rows_out, label_out, ts_out, weight_out, (int*)error);
    return launch_status();
}

int pin_train_gather_packed_split(const float* packed_pool, int64_t pool_rows, const int64_t* index, int64_t n_index,
                                  const int64_t* new_idx, int64_t new_count, const int64_t* index_new,
                                  const PinTrainCfg* cfg, float* rows_out, float* label_out, int64_t* ts_out,
                                  float* weight_out, int32_t* error, void* stream) {
    if (!cfg || n_index < 0 || n_index > cfg->n_main) return PIN_ERR_ARG;
    if (n_index < cfg->n_main && (!new_idx || !index_new || new_count < 1)) return PIN_ERR_ARG;
    if (n_index > 0 && !index) return PIN_ERR_ARG;
    const int rc = gather_packed_args(packed_pool, pool_rows, cfg, rows_out, label_out);
    if (rc != PIN_OK || cfg->n_main == 0) return rc;
    hipLaunchKernelGGL(k_train_gather_packed, grid_for(cfg->n_main), dim3(kTBlock), 0, as_stream(stream),
                       (const float4*)packed_pool, pool_rows, index, n_index, new_idx, new_count, index_new, *cfg,
                       rows_out, label_out, ts_out, weight_out, (int*)error);
    return launch_status();
}

int pin_train_gather_packed_draw(const float* packed_pool, int64_t pool_rows, int64_t n_hist, const int64_t* new_idx,
                                 int64_t new_count, uint64_t seed, uint64_t counter, const PinTrainCfg* cfg,
                                 float* rows_out, float* label_out, int64_t* ts_out, float* weight_out, int32_t* error,
                                 void* stream) {
    if (!cfg || n_hist < 0 || n_hist > cfg->n_main) return PIN_ERR_ARG;
    if (n_hist < cfg->n_main && (!new_idx || new_count < 1)) return PIN_ERR_ARG;
    const int rc = gather_packed_args(packed_pool, pool_rows, cfg, rows_out, label_out);
    if (rc != PIN_OK || cfg->n_main == 0) return rc;
    // the key on the host: one 64-bit mix of seed and counter per call
    auto hmix = [](uint64_t z) {
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    const BatchDraw dr{hmix(seed ^ hmix(counter)), 1};
    hipLaunchKernelGGL(k_train_gather_packed, grid_for(cfg->n_main), dim3(kTBlock), 0, as_stream(stream),
                       (const float4*)packed_pool, pool_rows, (const int64_t*)nullptr, n_hist, new_idx, new_count,
                       (const int64_t*)nullptr, *cfg, rows_out, label_out, ts_out, weight_out, (int*)error, dr);
    return launch_status();
}

int pin_train_gather(const float* coord_pool, const float* label_pool, const int64_t* ts_pool,
                     const float* weight_pool, int64_t pool_rows, const int64_t* index, const PinTrainCfg* cfg,
                     float* rows_out, float* label_out, int64_t* ts_out, float* weight_out, int32_t* error,
                     void* stream) {
    if (!cfg || cfg->n_main < 0 || cfg->n_stencil < 0 || cfg->decimation < 1) return PIN_ERR_ARG;
    if (cfg->n_stencil > 0 && (cfg->n_stencil - 1) * (int64_t)cfg->decimation >= cfg->n_main) return PIN_ERR_ARG;
    const int64_t rows = cfg->n_main + 6 * cfg->n_stencil;
    if (rows == 0) return PIN_OK;
    if (!coord_pool || !label_pool || !index || !rows_out || !label_out || (ts_pool && !ts_out) ||
        (weight_pool && !weight_out) || pool_rows < 1)
        return PIN_ERR_ARG;
    hipLaunchKernelGGL(k_train_gather, grid_for(cfg->n_main), dim3(kTBlock), 0, as_stream(stream), coord_pool,
                       label_pool, ts_pool, weight_pool, pool_rows, index, *cfg, rows_out, label_out, ts_out,
                       weight_out, (int*)error);
    return launch_status();
}

int pin_train_forward(const PinHash* hash, const PinGrid* grid, const PinPoints* pts, const PinMlp* mlp,
                      const float* coord, const int64_t* ts, const PinTrainCfg* cfg, const PinTrainState* st,
                      void* stream) {
    if (!pts || !mlp || !cfg || !st || !coord || !st->ids || !st->weights || !st->x || !st->sdf) return PIN_ERR_ARG;
    if ((!hash && !grid) || cfg->n_main < 0 || cfg->n_stencil < 0 || cfg->decimation < 1) return PIN_ERR_ARG;
    if (cfg->nn_k < 1 || cfg->nn_k > kK) return PIN_ERR_UNSUPPORTED;
    const int64_t rows = cfg->n_main + 6 * cfg->n_stencil;
    const bool dx = (cfg->flags & PIN_TRAIN_DX) != 0;
    // PIN_TRAIN_DX needs the matrix-core image in both decoding modes: the backward takes each
    // row's (weighted_first) or each neighbour's (masks) input gradient from it -- rejected here,
    // before the forward overwrites st.x, as pin_train_backward would reject it after
    if (dx && !mlp->packed) return PIN_ERR_ARG;
    const bool eik = (cfg->flags & PIN_TRAIN_EIK) != 0;
    if (eik && (dx || cfg->n_stencil != 0 || !st->eik_coef || !st->eik_vec)) return PIN_ERR_ARG;
    if (rows == 0) return PIN_OK;
    auto s = as_stream(stream);
    if (eik) {
        const bool wf = cfg->weighted_first != 0;
        if (grid) {
            if (wf) hipLaunchKernelGGL(k_train_forward_eik_grid<true>, grid_for(rows), dim3(kTBlock), 0, s, *grid, *pts,
                                       *mlp, coord, ts, *cfg, *st, 1);
            else hipLaunchKernelGGL(k_train_forward_eik_grid<false>, grid_for(rows), dim3(kTBlock), 0, s, *grid, *pts,
                                    *mlp, coord, ts, *cfg, *st, 1);
        } else {
            if (wf) hipLaunchKernelGGL(k_train_forward_eik_hash<true>, grid_for(rows), dim3(kTBlock), 0, s, *hash, *pts,
                                       *mlp, coord, ts, *cfg, *st, 1);
            else hipLaunchKernelGGL(k_train_forward_eik_hash<false>, grid_for(rows), dim3(kTBlock), 0, s, *hash, *pts,
                                    *mlp, coord, ts, *cfg, *st, 1);
        }
        return launch_status();
    }
#define PIN_LAUNCH_FWD(KERNEL, SRC)                                                                             \
    do {                                                                                                        \
        if (dx && cfg->weighted_first)                                                                          \
            hipLaunchKernelGGL((KERNEL<true, true>), grid_for(rows), dim3(kTBlock), 0, s, *SRC, *pts, *mlp,      \
                               coord, ts, *cfg, *st);                                                           \
        else if (dx && mlp->packed && kTrainNwfMf) /* per-neighbour: matrix-core decodes, masks saved */         \
            hipLaunchKernelGGL((KERNEL<false, true, true>), grid_for(rows), dim3(kTBlock), 0, s, *SRC, *pts,     \
                               *mlp, coord, ts, *cfg, *st);                                                     \
        else if (dx) /* per-neighbour: the f32 decode saves each neighbour's ReLU masks */                      \
            hipLaunchKernelGGL((KERNEL<false, false, true>), grid_for(rows), dim3(kTBlock), 0, s, *SRC, *pts,    \
                               *mlp, coord, ts, *cfg, *st);                                                     \
        else if (cfg->weighted_first && mlp->packed && kTrainFwdMf)                                             \
            hipLaunchKernelGGL((KERNEL<true, true, false>), grid_for(rows), dim3(kTBlock), 0, s, *SRC, *pts,     \
                               *mlp, coord, ts, *cfg, *st);                                                     \
        else if (cfg->weighted_first)                                                                           \
            hipLaunchKernelGGL((KERNEL<true, false>), grid_for(rows), dim3(kTBlock), 0, s, *SRC, *pts, *mlp,     \
                               coord, ts, *cfg, *st);                                                           \
        else                                                                                                    \
            hipLaunchKernelGGL((KERNEL<false, false>), grid_for(rows), dim3(kTBlock), 0, s, *SRC, *pts, *mlp,    \
                               coord, ts, *cfg, *st);                                                           \
    } while (0)
    if (grid && (cfg->flags & PIN_TRAIN_PAIR) && cfg->weighted_first && mlp->packed && (dx || kTrainFwdMf)) {
        // small batch: two lanes per row (k_train_forward_grid's PAIR)
        if (dx) hipLaunchKernelGGL((k_train_forward_grid<true, true, true, true>), grid_for(2 * rows), dim3(kTBlock), 0,
                                   s, *grid, *pts, *mlp, coord, ts, *cfg, *st);
        else hipLaunchKernelGGL((k_train_forward_grid<true, true, false, true>), grid_for(2 * rows), dim3(kTBlock), 0,
                                s, *grid, *pts, *mlp, coord, ts, *cfg, *st);
    } else if (grid) {
        PIN_LAUNCH_FWD(k_train_forward_grid, grid);
    } else {
        PIN_LAUNCH_FWD(k_train_forward_hash, hash);
    }
#undef PIN_LAUNCH_FWD
    return launch_status();
}

int pin_train_backward(const PinPoints* pts, const PinMlp* mlp, const float* label, const PinTrainCfg* cfg,
                       const PinTrainState* st, float* grad_features, float* mlp_grad, void* workspace,
                       double* loss_out, void* stream) {
    if (!pts || !mlp || !cfg || !st || !label || !st->ids || !st->weights || !st->x || !st->sdf) return PIN_ERR_ARG;
    if (cfg->nn_k < 1 || cfg->nn_k > kK) return PIN_ERR_UNSUPPORTED;
    const int64_t rows = cfg->n_main + 6 * cfg->n_stencil;
    if (rows == 0) return PIN_OK;
    if ((loss_out || mlp_grad) && !workspace) return PIN_ERR_ARG;
    if ((st->grad_fixed && (st->fixed_shift < 0 || st->fixed_shift > 62 || ((uintptr_t)st->grad_fixed & 15))) ||
        (st->cert_fixed && (st->cert_shift < 0 || st->cert_shift > 62)))
        return PIN_ERR_ARG;
    auto s = as_stream(stream);
    const dim3 g = grid_for(rows);
    const int64_t nblk = g.x;
    double* lpart = loss_out ? (double*)workspace : nullptr;
    float* mpart = mlp_grad ? (float*)((char*)workspace + nblk * kWaves * sizeof(double)) : nullptr;
    const int extra = (cfg->flags & PIN_TRAIN_EIK) ? 1 : 0;
    // the sorted-run scatter (feature_scatter_sorted) for large batches, which scatter straight
    // into the gradient; small ones (gradient replicas) keep the direct scatter: at 26K rows the
    // sort costs more than the replicas leave to save (backward 36 vs 28 us per SLAM-frame iteration)
    const bool sorted = PIN_SCAT_SORT && !(st->replicas > 1);
#define PIN_LAUNCH_BWD(WF, MG)                                                                                  \
    do {                                                                                                        \
        if (WF && sorted)                                                                                       \
            hipLaunchKernelGGL((k_train_backward<WF, MG, false, false, false, true>), g, dim3(kTBlock), 0, s,  \
                               *pts, *mlp, label, *cfg, *st, grad_features, mpart, lpart);                     \
        else                                                                                                    \
            hipLaunchKernelGGL((k_train_backward<WF, MG>), g, dim3(kTBlock), 0, s, *pts, *mlp, label, *cfg, *st, \
                               grad_features, mpart, lpart);                                                    \
    } while (0)
#define PIN_LAUNCH_BWD_EIK(WF, MG, MF)                                                                          \
    do {                                                                                                        \
        if (WF && sorted)                                                                                       \
            hipLaunchKernelGGL((k_train_backward<WF, MG, MF, true, false, true>), g, dim3(kTBlock), 0, s, *pts, \
                               *mlp, label, *cfg, *st, grad_features, mpart, lpart);                           \
        else                                                                                                    \
            hipLaunchKernelGGL((k_train_backward<WF, MG, MF, true>), g, dim3(kTBlock), 0, s, *pts, *mlp, label, \
                               *cfg, *st, grad_features, mpart, lpart);                                        \
    } while (0)
    if (cfg->flags & PIN_TRAIN_EIK) {
        if ((cfg->flags & PIN_TRAIN_DX) || cfg->n_stencil != 0 || !st->eik_coef || !st->eik_vec) return PIN_ERR_ARG;
        if (cfg->weighted_first) {
            if (mlp_grad) PIN_LAUNCH_BWD_EIK(true, true, false); else PIN_LAUNCH_BWD_EIK(true, false, false);
        } else {
            if (mlp_grad) PIN_LAUNCH_BWD_EIK(false, true, false);
            else if (mlp->packed) PIN_LAUNCH_BWD_EIK(false, false, true);
            else PIN_LAUNCH_BWD_EIK(false, false, false);
        }
    } else if (cfg->flags & PIN_TRAIN_DX) {
        if (mlp_grad || !mlp->packed) return PIN_ERR_UNSUPPORTED;
        if (cfg->weighted_first && sorted)
            hipLaunchKernelGGL((k_train_backward<true, false, true, false, false, true>), g, dim3(kTBlock), 0, s, *pts,
                               *mlp, label, *cfg, *st, grad_features, mpart, lpart);
        else if (cfg->weighted_first)
            hipLaunchKernelGGL((k_train_backward<true, false, true>), g, dim3(kTBlock), 0, s, *pts, *mlp, label, *cfg,
                               *st, grad_features, mpart, lpart);
        else if (sorted && PIN_NWF_SORT)   // per-neighbour masks, runs pre-summed in sorted order
            hipLaunchKernelGGL(k_train_backward_nwf_sorted, g, dim3(kTBlock), 0, s, *pts, *mlp, label, *cfg, *st,
                               grad_features, lpart);
        else
            hipLaunchKernelGGL((k_train_backward<false, false, true, false, true>), g, dim3(kTBlock), 0, s, *pts, *mlp,
                               label, *cfg, *st, grad_features, mpart, lpart);
    } else if (cfg->weighted_first) {
        if (mlp_grad && mlp->packed && sorted)   // a training decoder decoded on the matrix cores
            hipLaunchKernelGGL((k_train_backward<true, true, true, false, false, true>), g, dim3(kTBlock), 0, s, *pts,
                               *mlp, label, *cfg, *st, grad_features, mpart, lpart);
        else if (mlp_grad && mlp->packed)
            hipLaunchKernelGGL((k_train_backward<true, true, true>), g, dim3(kTBlock), 0, s, *pts, *mlp, label, *cfg,
                               *st, grad_features, mpart, lpart);
        else if (mlp_grad) PIN_LAUNCH_BWD(true, true);
        else PIN_LAUNCH_BWD(true, false);
    } else {
        if (mlp_grad) PIN_LAUNCH_BWD(false, true);
        else if (mlp->packed)
            hipLaunchKernelGGL((k_train_backward<false, false, true>), g, dim3(kTBlock), 0, s, *pts, *mlp, label, *cfg,
                               *st, grad_features, mpart, lpart);
        else PIN_LAUNCH_BWD(false, false);
    }
#undef PIN_LAUNCH_BWD
#undef PIN_LAUNCH_BWD_EIK
    if (grad_features && st->grad_fixed && st->replica_mode == 0) {   // deterministic mode
        const int64_t n = pts->rows * kF;
        const int64_t nb = (n + kTBlock - 1) / kTBlock;
        hipLaunchKernelGGL(k_fixed_reduce, dim3((unsigned)(nb < 2048 ? nb : 2048)), dim3(kTBlock), 0, s,
                           (long long*)st->grad_fixed, st->replicas > 1 ? st->replicas : 1, n, st->fixed_shift, 2,
                           grad_features);
    } else if (grad_features && st->grad_replicas && st->replicas > 1 && st->replica_mode == 0) {
        const int64_t n4 = pts->rows * kF / 4;
        const int64_t nb = (n4 + kTBlock - 1) / kTBlock;
        hipLaunchKernelGGL(k_replica_reduce, dim3((unsigned)(nb < 2048 ? nb : 2048)), dim3(kTBlock), 0, s,
                           (float4*)st->grad_replicas, st->replicas, n4, (float4*)grad_features);
    }
    if (mlp_grad)   // decoder gradients (+ the loss in one more block)
        hipLaunchKernelGGL(k_mlp_grad_final, dim3(kH / 4 + (loss_out ? 1 : 0)), dim3(kTBlock), 0, s, mpart, nblk, extra,
                           *mlp, mlp_grad, lpart, nblk * kWaves, loss_out);
    else if (loss_out)
        hipLaunchKernelGGL(k_loss_final, dim3(1), dim3(1024), 0, s, lpart, nblk * kWaves, loss_out);
    return launch_status();
}

int pin_adam_step(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n, const PinAdamStep* a,
                  void* stream) {
    if (!a || n < 0 || (n > 0 && (!param || !grad || !exp_avg || !exp_avg_sq))) return PIN_ERR_ARG;
    if (a->grad_stride != 8 && (a->grad_stride < 8 || n % 8)) return PIN_ERR_ARG;
    if (n == 0) return PIN_OK;
    if (((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) & 15) return PIN_ERR_ARG;
    hipLaunchKernelGGL(k_adam, grid_for((n + 3) / 4), dim3(kTBlock), 0, as_stream(stream), param, grad, exp_avg,
                       exp_avg_sq, n, *a);
    return launch_status();
}

}  // extern "C"
