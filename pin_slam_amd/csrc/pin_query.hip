// pin_query.hip -- neural-point query kernels for gfx950 (MI355X) and their C ABI.
//
// One lane owns one query.  The lane hashes its voxel once, then probes the Kc
// neighbour cells in chunks (all probes of a chunk in flight before their records
// are read), keeps the k nearest candidates in a register top-k, gathers the k
// feature rows (2 x 16 B loads each), and -- in the fused path -- evaluates the
// 11->64->1 decoder with its weights in scalar registers (wave-uniform loads) and
// the closed-form dSDF/dq.  See DESIGN.md for the roofline and data layout.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>

#include "pin_device.h"

// Per-neighbour decoder (weighted_first False) of the fused grid kernel as one f32-MFMA GEMM per
// neighbour slot (mlp_sdf_wave).  Off: measured 123 us vs 102 us on VALU for 262K queries -- the
// f32 MFMA runs at the packed-f32 VALU rate on gfx950 and an 11-input hidden unit needs ~4 VALU
// ops of post-processing (bias, ReLU, w2, mask) for ~5.5 packed FMAs saved.
#ifndef PIN_MLP_MFMA
#define PIN_MLP_MFMA 0
#endif

using namespace pin;

namespace {

inline dim3 grid_for(int64_t n) { return dim3((unsigned)((n + kBlock - 1) / kBlock)); }
inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline int launch_status() { return hipGetLastError() == hipSuccess ? PIN_OK : PIN_ERR_HIP; }

bool hash_ok(const PinHash* h) {
    return h && h->table && h->cells && h->num_cells > 0 && h->buffer_size > 0 && h->buffer_size < (1ll << 31) &&
           h->resolution > 0.f;
}
bool points_ok(const PinPoints* p) { return p && p->records && p->num_points >= 0; }

// ------------------------------------------------------------------ records
__global__ void __launch_bounds__(kBlock)
k_build_records(const float* __restrict__ pos, int64_t M, int32_t local, const int64_t* __restrict__ g2l,
                const int64_t* __restrict__ ts_create, const float* __restrict__ travel, int64_t cur_ts,
                float diff_local, const float* __restrict__ lpos, int64_t lrows, float4* __restrict__ out) {
    const int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (g >= M) return;
    const float x = pos[3 * g], y = pos[3 * g + 1], z = pos[3 * g + 2];
    int id = (int)g;
    if (local) {
        if (travel) {
            const float dtd = fabsf(travel[cur_ts] - travel[ts_create[g]]);
            if (!(dtd < diff_local)) id = -1;
        }
        if (id >= 0 && g2l) {
            const int64_t l = g2l[g];
            id = (int)l;
            if (l >= 0 && lpos && l < lrows) {
                const bool same = __float_as_int(lpos[3 * l]) == __float_as_int(x) &&
                                  __float_as_int(lpos[3 * l + 1]) == __float_as_int(y) &&
                                  __float_as_int(lpos[3 * l + 2]) == __float_as_int(z);
                if (!same) id |= PIN_RECORD_UNFAITHFUL;
            }
        }
    }
    out[g] = make_float4(x, y, z, __int_as_float(id));
}

// ------------------------------------------------------------------ hash rebuild
__global__ void __launch_bounds__(kBlock)
k_hash_rebuild(const float* __restrict__ pos, int64_t n, float res, int32_t* __restrict__ table, int64_t B) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint32_t s = base_slot(pos[3 * i], pos[3 * i + 1], pos[3 * i + 2], res, B);
    atomicMax(table + s, (int)i);  // last writer of the CPU reference = highest index
}

// ------------------------------------------------------------------ radius search
__global__ void __launch_bounds__(kBlock)
k_radius_search(const PinHash h, const float4* __restrict__ rec, const float* __restrict__ q, int64_t n,
                float* __restrict__ dist2_out, int64_t* __restrict__ idx_out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float qx = q[3 * i], qy = q[3 * i + 1], qz = q[3 * i + 2];
    const uint32_t B = (uint32_t)h.buffer_size;
    const uint32_t base = base_slot(qx, qy, qz, h.resolution, h.buffer_size);
    const int Kc = h.num_cells;
    for (int c = 0; c < Kc; ++c) {
        uint32_t s = base + (uint32_t)h.cells[c];
        s = s >= B ? s - B : s;
        int g = h.table[s];
        float d2 = h.max_valid_dist2;
        if (g >= 0) {
            const float4 r = rec[g];
            if (__float_as_int(r.w) == -1) {
                g = -1;  // time-filtered before the distance (neural_points.py:488)
            } else {
                d2 = dist2(r.x, r.y, r.z, qx, qy, qz);
                if (d2 > h.max_valid_dist2) g = -1;
            }
        }
        dist2_out[i * Kc + c] = d2;
        idx_out[i * Kc + c] = g;
    }
}

// ------------------------------------------------------------------ certainty
__global__ void __launch_bounds__(kBlock)
k_query_certainty(const PinHash h, const float4* __restrict__ rec, const float* __restrict__ cert,
                  const float* __restrict__ q, int64_t n, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float qx = q[3 * i], qy = q[3 * i + 1], qz = q[3 * i + 2];
    const uint32_t B = (uint32_t)h.buffer_size;
    const uint32_t base = base_slot(qx, qy, qz, h.resolution, h.buffer_size);
    float m = -INFINITY;
    for (int c = 0; c < h.num_cells; ++c) {
        uint32_t s = base + (uint32_t)h.cells[c];
        s = s >= B ? s - B : s;
        const int g = h.table[s];
        float val = 0.f;
        if (g >= 0) {
            const float4 r = rec[g];
            if (dist2(r.x, r.y, r.z, qx, qy, qz) <= h.max_valid_dist2) val = cert[g];
        }
        m = fmaxf(m, val);
    }
    out[i] = m;
}

// ------------------------------------------------------------------ fused SDF (+grad)
// Tracker / mesher inference: query_feature + Decoder.sdf + get_gradient in one pass.
// One neighbour of the top-k list, streamed: its record (position, id), decoder input
// x = [f, v] (v rotated after pgo), quaternion and certainty.  Invalid -> zeros.
struct NbInput {
    float x[kD];
    float pg[3];   // q - global position
    float4 quat;
    float cert;
};

template <bool PGO, bool CERT, class Src>
__device__ __forceinline__ void stream_neighbour(const Src& src, const PinPoints& p, int pay, bool valid, float qx,
                                                 float qy, float qz, NbInput& o) {
#if defined(PIN_PROF_STAGE) && PIN_PROF_STAGE == 2
    // profiling variant: no record re-gather (wrong positions, same instruction stream otherwise)
    const float4 r = make_float4(qx + 0.1f, qy - 0.1f, qz + 0.05f * (float)(pay & 7), __int_as_float(pay));
#else
    const float4 r = src.record(pay);
#endif
    const int raw = __float_as_int(r.w);
    const int64_t id = valid ? (raw & kIdMask) : 0;
    float4 f0, f1;
#if defined(PIN_PROF_STAGE) && PIN_PROF_STAGE == 3
    // profiling variant: no feature gathers
    f0 = make_float4(r.x * 0.01f, r.y * 0.01f, r.z * 0.01f, 0.02f);
    f1 = make_float4(r.y * 0.02f, r.z * 0.02f, r.x * 0.03f, -0.02f);
#else
    src.features(pay, id, f0, f1);
#endif
    o.pg[0] = qx - r.x;
    o.pg[1] = qy - r.y;
    o.pg[2] = qz - r.z;
    float v0 = o.pg[0], v1 = o.pg[1], v2 = o.pg[2];
    if (valid && (raw & PIN_RECORD_UNFAITHFUL)) {  // global2local quirk: local position differs
        v0 = qx - p.positions[3 * id];
        v1 = qy - p.positions[3 * id + 1];
        v2 = qz - p.positions[3 * id + 2];
    }
    o.quat = make_float4(1.f, 0.f, 0.f, 0.f);
    if (PGO) {
        o.quat = ((const float4*)p.orientations)[id];
        quat_rotate_passive(o.quat, v0, v1, v2);
    }
    o.cert = CERT ? src.certainty(pay, id) : 0.f;
    const float f[kD] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w, v0, v1, v2};
#pragma unroll
    for (int d = 0; d < kD; ++d) o.x[d] = valid ? f[d] : 0.f;
    if (!valid) o.cert = 0.f;
}

// Everything after the candidate scan: IDW weights, streamed neighbour inputs, decoder,
// closed-form gradient, outputs.  Used by the fused kernels and by the split epilogue.
template <bool WF, bool PGO, bool GRAD, class Src, bool MF = false>
__device__ __forceinline__ void query_sdf_epilogue(const Src& src, const PinPoints& p, const MlpW& m, float qx,
                                                   float qy, float qz, const TopK& tk, int nn, int64_t i, int nn_k,
                                                   int zero_empty, float* __restrict__ sdf_out,
                                                   float* __restrict__ grad_out, int* __restrict__ nn_out,
                                                   float* __restrict__ cert_out, float* __restrict__ std_out) {
    // IDW weights from the top-k distances alone (neural_points.py:618-632)
    float u[kK];
    float S = 0.f;
#pragma unroll
    for (int j = 0; j < kK; ++j) {
        u[j] = (j < nn_k && tk.g[j] >= 0) ? 1.0f / (tk.d[j] + kIdwEps) : 0.f;
        S = S + u[j];
    }
    const float invS = nn > 0 ? 1.f / S : 0.f;
    const bool want_cert = cert_out != nullptr;

    float cert = 0.f;
    float sdf = 0.f, std_v = 0.f;
    float gq[3] = {0.f, 0.f, 0.f};
    if constexpr (WF) {
        // One streamed pass over the neighbours accumulates
        //   x  = sum_j w_j x_j                      (neural_points.py:660-662)
        //   J  = sum_j x_j (x) c_j,  C = sum_j c_j,  c_j = -2 u_j^2 (q - p_j) / S
        //        so that sum_j (a_j - abar) c_j = J^T gx - (gx . x) C  with a_j = gx . x_j
        //        (the same un-centred form autograd evaluates for d(u/S)/du)
        //   Wr = sum_j w_j R_j  (pgo; the scalar sum_j w_j otherwise)
        float x[kD], J[kD][3], C[3] = {0.f, 0.f, 0.f}, Wr[3][3];
#pragma unroll
        for (int d = 0; d < kD; ++d) { x[d] = 0.f; J[d][0] = J[d][1] = J[d][2] = 0.f; }
#pragma unroll
        for (int a = 0; a < 3; ++a) Wr[a][0] = Wr[a][1] = Wr[a][2] = 0.f;
#pragma unroll
        for (int j = 0; j < kK; ++j) {
            // neighbours stream in two groups of four: bounds the registers held by gathers
            // in flight while keeping four lines outstanding per lane
            if (j && j % PIN_NB_GROUP == 0) __builtin_amdgcn_sched_barrier(0);
            const bool valid = u[j] > 0.f;
            NbInput in;
            if (want_cert) stream_neighbour<PGO, true>(src, p, tk.g[j], valid, qx, qy, qz, in);
            else stream_neighbour<PGO, false>(src, p, tk.g[j], valid, qx, qy, qz, in);
            const float w = valid && nn > 0 ? u[j] / S : 0.f;
            cert = cert + in.cert * w;
#pragma unroll
            for (int d = 0; d < kD; ++d) x[d] = x[d] + in.x[d] * w;
            if (GRAD) {
                const float cu = valid ? -2.f * u[j] * u[j] * invS : 0.f;
                const float c3[3] = {cu * in.pg[0], cu * in.pg[1], cu * in.pg[2]};
#pragma unroll
                for (int a = 0; a < 3; ++a) C[a] += c3[a];
#pragma unroll
                for (int d = 0; d < kD; ++d) {
#pragma unroll
                    for (int a = 0; a < 3; ++a) J[d][a] = fmaf(in.x[d], c3[a], J[d][a]);
                }
                if (PGO) {
                    float R[3][3];
                    quat_rotmat(in.quat, R);
#pragma unroll
                    for (int a = 0; a < 3; ++a)
#pragma unroll
                        for (int b = 0; b < 3; ++b) Wr[a][b] = fmaf(w, R[a][b], Wr[a][b]);
                } else {
                    Wr[0][0] += w;
                }
            }
        }
        float gx[kD];
#if defined(PIN_PROF_STAGE) && PIN_PROF_STAGE == 4
        // profiling variant: no decoder (a linear stand-in with the same outputs' shapes)
        sdf = 0.f;
#pragma unroll
        for (int d = 0; d < kD; ++d) { gx[d] = 0.01f * (float)(d + 1); sdf = fmaf(x[d], gx[d], sdf); }
#else
        if constexpr (MF) sdf = mlp_sdf_mfma16<GRAD, 0, kD, PGO>(m, x, gx);   // after PGO: tile-outer GEMM order
        else sdf = mlp_sdf<GRAD, 0, kD>(m, x, gx);
#endif
        if (nn == 0 && zero_empty) sdf = 0.f;
        if (GRAD && nn > 0) {
            float abar = 0.f;
#pragma unroll
            for (int d = 0; d < kD; ++d) abar = fmaf(gx[d], x[d], abar);
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                float s = -abar * C[a];
#pragma unroll
                for (int d = 0; d < kD; ++d) s = fmaf(gx[d], J[d][a], s);
                gq[a] = s;
            }
            if (PGO) {
#pragma unroll
                for (int a = 0; a < 3; ++a)
#pragma unroll
                    for (int b = 0; b < 3; ++b) gq[a] = fmaf(Wr[a][b], gx[kF + b], gq[a]);
            } else {
#pragma unroll
                for (int a = 0; a < 3; ++a) gq[a] = fmaf(Wr[0][0], gx[kF + a], gq[a]);
            }
        }
    } else {
        // per-neighbour decoding, weighted mean / std (utils/tracker.py:245-249);
        // gradient = sum_j sk_j c_j - mean C + sum_j w_j R_j gv_j
        float sk[kK];
        float w[kK];
        float A[3] = {0.f, 0.f, 0.f}, C[3] = {0.f, 0.f, 0.f}, G[3] = {0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < kK; ++j) {
            // matrix-core decoder: one neighbour's gathers in flight at a time (hoisting the
            // next neighbours' gathers over the GEMMs spills)
            if (MF && j) __builtin_amdgcn_sched_barrier(0);
            const bool valid = u[j] > 0.f;
            NbInput in;
            if (want_cert) stream_neighbour<PGO, true>(src, p, tk.g[j], valid, qx, qy, qz, in);
            else stream_neighbour<PGO, false>(src, p, tk.g[j], valid, qx, qy, qz, in);
            w[j] = valid && nn > 0 ? u[j] / S : 0.f;
            cert = cert + in.cert * w[j];
            sk[j] = 0.f;
            float g3[3];
            if constexpr (MF) {   // the wave's 64 neighbour-j decodes on the f16 matrix cores
                const float v = mlp_sdf_mfma16<GRAD, kF, 3>(m, in.x, g3);
                if (!valid) continue;
                sk[j] = v;
            } else if (m.xs) {   // the wave's 64 neighbour-j decodes as one MFMA GEMM (all lanes take part)
                const float v = mlp_sdf_wave<GRAD, kF, 3>(m, in.x, g3);
                if (!valid) continue;
                sk[j] = v;
            } else {
                if (!valid) continue;
                sk[j] = mlp_sdf<GRAD, kF, 3>(m, in.x, g3);
            }
            if (GRAD) {
                float r0 = g3[0], r1 = g3[1], r2 = g3[2];
                if (PGO) quat_rotate_active(in.quat, g3[0], g3[1], g3[2], r0, r1, r2);
                G[0] = fmaf(w[j], r0, G[0]);
                G[1] = fmaf(w[j], r1, G[1]);
                G[2] = fmaf(w[j], r2, G[2]);
                const float cu = -2.f * u[j] * u[j] * invS;
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    const float c = cu * in.pg[a];
                    C[a] += c;
                    A[a] = fmaf(sk[j], c, A[a]);
                }
            }
        }
        float mean = 0.f;
#pragma unroll
        for (int j = 0; j < kK; ++j) mean = mean + sk[j] * w[j];
        float var = 0.f;
#pragma unroll
        for (int j = 0; j < kK; ++j) {
            const float dv = sk[j] - mean;
            var = var + w[j] * (dv * dv);
        }
        sdf = mean;
        std_v = sqrtf(var);
        if (GRAD && nn > 0) {
#pragma unroll
            for (int a = 0; a < 3; ++a) gq[a] = A[a] - mean * C[a] + G[a];
        }
    }
    if (i < 0) return;   // a lane that only kept the wave whole for the MFMA decoder
    if (sdf_out) sdf_out[i] = sdf;
    if (GRAD && grad_out) {
        grad_out[3 * i] = gq[0];
        grad_out[3 * i + 1] = gq[1];
        grad_out[3 * i + 2] = gq[2];
    }
    if (nn_out) nn_out[i] = nn;
    if (cert_out) cert_out[i] = cert;
    if (std_out) std_out[i] = std_v;
}

template <bool WF, bool PGO, bool GRAD, class Src, bool MF = false>
__device__ __forceinline__ void query_sdf_body(const Src& src, const PinPoints& p, const MlpW& m, float qx, float qy,
                                               float qz, int64_t i, int nn_k, int zero_empty,
                                               float* __restrict__ sdf_out, float* __restrict__ grad_out,
                                               int* __restrict__ nn_out, float* __restrict__ cert_out,
                                               float* __restrict__ std_out) {
    // i < 0: no query (the lane only completes its wave); nothing is written for it
    TopK tk;
    tk.init();
    const int nn = src.template scan<Src::kChunk>(qx, qy, qz, tk);
    resolve_ties(src, qx, qy, qz, nn_k, nn, tk);   // the reference's neighbour set at equal distances
#if defined(PIN_PROF_STAGE) && PIN_PROF_STAGE == 1
    // profiling variant: candidate scan only (the top-k kept live through one output)
    if (i >= 0) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < kK; ++j) s += tk.d[j] + (float)tk.g[j];
        sdf_out[i] = s;
        nn_out[i] = nn;
    }
    return;
#endif
    query_sdf_epilogue<WF, PGO, GRAD, Src, MF>(src, p, m, qx, qy, qz, tk, nn, i, nn_k, zero_empty, sdf_out,
                                               grad_out, nn_out, cert_out, std_out);
}

// MF: decoder on the f16 matrix cores (whole waves run; lanes past n compute query 0 unwritten).
template <bool WF, bool PGO, bool GRAD, bool MF>
__global__ void __launch_bounds__(kBlock)
k_query_sdf(const PinHash h, const PinPoints p, const PinMlp m, const float* __restrict__ q, int64_t n, int nn_k,
            int zero_empty, float* __restrict__ sdf_out, float* __restrict__ grad_out, int* __restrict__ nn_out,
            float* __restrict__ cert_out, float* __restrict__ std_out) {
    __shared__ float s_mlp[MF ? 1 : kWSize];
    __shared__ uint4 s_pk[MF ? kPkBytes / 16 : 1];
    const MlpW mw = stage_decoder<MF>(m, s_mlp, s_pk);
    const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if ((t & ~(int64_t)63) >= n) return;   // whole waves (the MFMA decoder, resolve_ties): lanes past n run query 0
    const int64_t i = t < n ? t : -1, iq = t < n ? t : 0;
    const HashSource src(h, p);
    query_sdf_body<WF, PGO, GRAD, HashSource, MF>(src, p, mw, q[3 * iq], q[3 * iq + 1], q[3 * iq + 2], i, nn_k,
                                                  zero_empty, sdf_out, grad_out, nn_out, cert_out, std_out);
}

#ifndef PIN_SDF_WAVES
#define PIN_SDF_WAVES 2   // waves per SIMD the fused grid kernel is compiled for (VGPR budget)
#endif
#ifndef PIN_SDF_WAVES_NWF
#define PIN_SDF_WAVES_NWF PIN_SDF_WAVES   // the same for per-neighbour decoding
#endif
#ifndef PIN_SDF_WAVES_PGO
#define PIN_SDF_WAVES_PGO 2   // after pose-graph optimisation (quaternion-rotated neighbour vectors):
#endif                        // 1 wave/SIMD at 256 VGPRs + 37 AGPRs before

// q4 != NULL: the queries pre-sorted by pin_query_sort, {x, y, z, bits(original index)} each
// (one coalesced 16-B load, no order -> coordinate dependency); otherwise q [n,3] processed in
// `order` (or input order).
// MF: decoder on the f16 matrix cores (mlp_sdf_mfma16, m.packed from pin_mlp_pack).
template <bool WF, bool PGO, bool GRAD, bool FAT, bool MF>
__global__ void __launch_bounds__(kBlock)
__attribute__((amdgpu_waves_per_eu(PGO ? PIN_SDF_WAVES_PGO
                                        : (!MF && (!GRAD || !WF)) ? 4   // the SDF-only / f32 per-neighbour forms fit 128
                                        : (WF ? PIN_SDF_WAVES : PIN_SDF_WAVES_NWF))))
k_query_sdf_grid(const PinGrid g, const PinPoints p, const PinMlp m, const float* __restrict__ q,
                 const float4* __restrict__ q4, int64_t n, int nn_k, int zero_empty, float* __restrict__ sdf_out,
                 float* __restrict__ grad_out, int* __restrict__ nn_out, float* __restrict__ cert_out,
                 float* __restrict__ std_out, const int* __restrict__ order, int out_slot) {
    __shared__ float s_mlp[MF ? 1 : kWSize];
    __shared__ uint4 s_pk[MF ? kPkBytes / 16 : 1];
    MlpW mw = stage_decoder<MF>(m, s_mlp, s_pk);
    const int64_t t = xcd_block() * kBlock + threadIdx.x;
#if PIN_MLP_MFMA
    __shared__ float s_xs[kBlock / 64][64 * kWRow];
    if (!WF && !MF) mw.xs = s_xs[threadIdx.x >> 6];
#endif
    // whole waves (the MFMA decoders, resolve_ties): lanes past n run query 0 and write nothing
    if ((t & ~(int64_t)63) >= n) return;
    const int64_t tt = t < n ? t : 0;
    float qx, qy, qz;
    int64_t i;
    if (q4) {
        const float4 v = q4[tt];
        qx = v.x; qy = v.y; qz = v.z;
        const int iw = __float_as_int(v.w);
        i = (t < n && iw >= 0 && iw < n) ? iw : -1;
    } else {
        i = t < n ? (order ? order[t] : t) : -1;
        const int64_t iq = i >= 0 ? i : 0;
        qx = q[3 * iq]; qy = q[3 * iq + 1]; qz = q[3 * iq + 2];
    }
    // out_slot: outputs at the processing position (tile order, coalesced stores) instead of the
    // query's own index -- for consumers that reduce over the queries (the tracker) or read q4
    if (out_slot && i >= 0) i = t;
    const GridSource<FAT> src(g, p);
    query_sdf_body<WF, PGO, GRAD, GridSource<FAT>, MF>(src, p, mw, qx, qy, qz, i, nn_k, zero_empty, sdf_out, grad_out,
                                                       nn_out, cert_out, std_out);
}

// Query tiling: one counting-sort pass of the queries into <= kMaxTiles spatial tiles of the grid
// box (cubes of 2^shift cells; the host picks the smallest shift >= 3 with <= kMaxTiles tiles).  Random
// batches are then processed tile by tile: a block's gathers share lines and, with xcd_block(),
// each XCD's L2 holds one region of the map.  Order inside a tile is arbitrary (it depends on
// atomic arrival); every query's outputs still go to its own index, so results are unchanged.
//
//   k_tile_rank   per block: LDS tile histogram (the returning LDS atomic is the query's rank in
//                 its tile within the block), then one returning global atomic per (block, tile)
//                 reserves the block's run inside the tile: off = run + rank, stored per query
//   k_tile_place  per block: exclusive scan of the tile totals -> tile bases; each query
//                 lands at base[tile] + off.  The last block to finish zeroes the totals again.
// Workspace state (PIN_ORDER_STATE_BYTES): tile totals + a done counter, zero before the first
// call and zero again after each call; then n int2 (tile, off).
// Tile capacity: 4,096 tiles (16x16-cell columns on the 1000x1000 surface: ~one wave per tile)
// for batches below 1M rows; 16,384 for larger ones (the mapper's 1.68M rows over the 2000x2000
// map: 16x16-cell columns instead of 32x32, ~107 rows per tile -- mapper +6 % measured; at 262K
// queries the query kernel gains 2 us but the sort's larger histograms cost 4.5 us).
#ifndef PIN_MAX_TILES
#define PIN_MAX_TILES 4096
#endif
#ifndef PIN_MAX_TILES_LARGE
#define PIN_MAX_TILES_LARGE 16384
#endif
constexpr int kMaxTiles = PIN_MAX_TILES;
constexpr int kMaxTilesLarge = PIN_MAX_TILES_LARGE;
constexpr int64_t kLargeBatch = 1 << 20;
constexpr int kPartThreads = 1024;
static_assert(kMaxTiles % kPartThreads == 0 && kMaxTilesLarge % kPartThreads == 0,
              "tile capacity must be a multiple of the block");

struct TileMap {
    int64_t ox, oy, oz;
    float inv_res;   // ordering only: a reciprocal is fine here
    int shift, ntx, nty, ntz, ntiles;
};

__device__ __forceinline__ int tile_of(float x, float y, float z, const TileMap& t) {
    auto axis = [&](float v, int64_t o, int nt) -> int {
        const int64_t c = ((int64_t)floorf(v * t.inv_res) - o) >> t.shift;
        return (int)(c < 0 ? 0 : (c >= nt ? nt - 1 : c));
    };
    return (axis(z, t.oz, t.ntz) * t.nty + axis(y, t.oy, t.nty)) * t.ntx + axis(x, t.ox, t.ntx);
}

// Both kernels issue every load of a thread before using any (one memory round trip per phase).
template <int PER, int MAXT>
__global__ void __launch_bounds__(kPartThreads)
k_tile_rank(const float* __restrict__ q, int64_t n, TileMap t, int* __restrict__ tot, int2* __restrict__ tk) {
    constexpr int kTpt = MAXT / kPartThreads;   // tiles per thread in the atomic and scan phases
    static_assert(4 * MAXT <= 160 * 1024 / 2, "k_tile_rank's LDS histogram: gfx950 has 160 KB per CU (two blocks)");
    __shared__ int h[MAXT];
    const int k = threadIdx.x;
#pragma unroll
    for (int j = 0; j < kTpt; ++j) h[k + j * kPartThreads] = 0;
    const int64_t lo = (int64_t)blockIdx.x * PER * kPartThreads + k;
    float x[PER], y[PER], z[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int64_t i = lo + (int64_t)u * kPartThreads;
        const int64_t j = i < n ? i : 0;
        x[u] = q[3 * j];
        y[u] = q[3 * j + 1];
        z[u] = q[3 * j + 2];
    }
    int tile[PER], rank[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) tile[u] = lo + (int64_t)u * kPartThreads < n ? tile_of(x[u], y[u], z[u], t) : -1;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PER; ++u) rank[u] = tile[u] >= 0 ? atomicAdd(h + tile[u], 1) : 0;
    __syncthreads();
    // this block's run inside each tile (independent returning atomics); every block visits the
    // tiles from its own starting point, so the blocks' same-address atomics on a line of the totals
    // arrive spread over time instead of all blocks on the first line at once
    const int rot = (int)((blockIdx.x * 1237u) & (MAXT - 1)) & ~63;
    int run[kTpt];
#pragma unroll
    for (int j = 0; j < kTpt; ++j) {
        const int tt = (k + j * kPartThreads + rot) & (MAXT - 1);
        const int c = h[tt];
        run[j] = c ? atomicAdd(tot + tt, c) : 0;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kTpt; ++j) h[(k + j * kPartThreads + rot) & (MAXT - 1)] = run[j];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int64_t i = lo + (int64_t)u * kPartThreads;
        if (tile[u] >= 0) tk[i] = make_int2(tile[u], h[tile[u]] + rank[u]);
    }
}

template <int PER, int MAXT>
__global__ void __launch_bounds__(kPartThreads)
k_tile_place(const float* __restrict__ q, int64_t n, int ntiles, int* __restrict__ tot, unsigned* __restrict__ done,
             const int2* __restrict__ tk, float4* __restrict__ q4, int* __restrict__ order) {
    constexpr int kTpt = MAXT / kPartThreads;
    static_assert(4 * MAXT + 4 * (kPartThreads / 64) + 4 <= 160 * 1024 / 2,
                  "k_tile_place's LDS tile bases: gfx950 has 160 KB per CU (two blocks); other targets have 64 KB");
    __shared__ int base[MAXT];
    __shared__ int wsum[kPartThreads / 64];
    __shared__ int last;
    const int k = threadIdx.x;
    const int64_t lo = (int64_t)blockIdx.x * PER * kPartThreads + k;
    int v[kTpt], sum = 0;   // thread k owns tiles kTpt*k .. kTpt*k + kTpt-1 (consecutive)
#pragma unroll
    for (int j = 0; j < kTpt; ++j) {
        v[j] = kTpt * k + j < ntiles ? tot[kTpt * k + j] : 0;
        sum += v[j];
    }
    int2 e[PER];
    float x[PER], y[PER], z[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int64_t i = lo + (int64_t)u * kPartThreads;
        const int64_t j = i < n ? i : 0;
        e[u] = tk[j];
        if (q4) {
            x[u] = q[3 * j];
            y[u] = q[3 * j + 1];
            z[u] = q[3 * j + 2];
        }
    }
    // exclusive scan of the tile totals
    int incl = sum;
    for (int o = 1; o < 64; o <<= 1) {
        const int w = __shfl_up(incl, o);
        if ((k & 63) >= o) incl += w;
    }
    if ((k & 63) == 63) wsum[k >> 6] = incl;
    __syncthreads();
    // after the barrier every wave of the block has its totals in hand: count the block as done
    // (the returning atomic's latency overlaps the placement below; its value is used at the end)
    unsigned ticket = 0;
    if (k == 0) ticket = atomicInc(done, gridDim.x - 1);   // wraps back to 0 after the last block
    int run = incl - sum;
    for (int w = 0; w < (k >> 6); ++w) run += wsum[w];
#pragma unroll
    for (int j = 0; j < kTpt; ++j) {
        base[kTpt * k + j] = run;
        run += v[j];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int64_t i = lo + (int64_t)u * kPartThreads;
        const int64_t pos = (int64_t)base[e[u].x & (MAXT - 1)] + e[u].y;
        if (i >= n || pos < 0 || pos >= n) continue;   // pos: only a workspace whose state was not zeroed
        if (q4) q4[pos] = make_float4(x[u], y[u], z[u], __int_as_float((int)i));
        if (order) order[pos] = (int)i;
    }
    // every block read the totals before its atomicInc: the last one clears them for the next call
    if (k == 0) last = ticket == gridDim.x - 1;
    __syncthreads();
    if (last) {
#pragma unroll
        for (int j = 0; j < kTpt; ++j) tot[k + j * kPartThreads] = 0;
    }
}

// host: tile map of a grid box with at most maxt tiles
TileMap tile_map(const PinGrid& g, int maxt) {
    TileMap t;
    t.ox = g.dims.ox;
    t.oy = g.dims.oy;
    t.oz = g.dims.oz;
    t.inv_res = 1.0f / g.resolution;
    const int64_t ex = 4ll * g.dims.nbx, ey = 4ll * g.dims.nby, ez = 4ll * g.dims.nbz;
    int sh = 3;
    for (;; ++sh) {
        const int64_t nx = (ex + (1ll << sh) - 1) >> sh, ny = (ey + (1ll << sh) - 1) >> sh,
                      nz = (ez + (1ll << sh) - 1) >> sh;
        if (nx * ny * nz <= maxt) {
            t.ntx = (int)nx;
            t.nty = (int)ny;
            t.ntz = (int)nz;
            break;
        }
    }
    t.shift = sh;
    t.ntiles = t.ntx * t.nty * t.ntz;
    return t;
}

// the tile sort of q: q4 (may be NULL) = {x, y, z, bits(i)} in tile order, order (may be NULL) =
// the indices in tile order; workspace = pin_query_order_workspace_bytes(n) with zeroed state.
// 4 queries per thread up to 512K queries (64 blocks at 256K), 16 beyond (<= ~256 blocks at
// 4M): few blocks keep the same-address atomics on the tile totals few.
int sort_queries(const PinGrid& g, const float* q, int64_t n, float4* q4, int* order, void* workspace,
                 hipStream_t s) {
    const bool large = n >= kLargeBatch;
    const TileMap t = tile_map(g, large ? kMaxTilesLarge : kMaxTiles);
    char* ws = (char*)workspace;
    int* tot = (int*)ws;
    // the done counter sits past the largest capacity's totals (either capacity leaves its
    // totals zero, so calls of both sizes may share a workspace)
    unsigned* done = (unsigned*)(ws + 4 * (kMaxTilesLarge > kMaxTiles ? kMaxTilesLarge : kMaxTiles));
    static_assert(4 * kMaxTilesLarge + 64 <= PIN_ORDER_STATE_BYTES && 4 * kMaxTiles + 64 <= PIN_ORDER_STATE_BYTES,
                  "order workspace state too small");
    int2* tk = (int2*)(ws + PIN_ORDER_STATE_BYTES);
    // the placement does not depend on the ranking's blocks: it runs 2 queries per thread (more
    // blocks in flight for its scattered 16-B stores)
#ifndef PIN_PLACE_PER
#define PIN_PLACE_PER 2
#endif
#ifndef PIN_RANK_PER
#define PIN_RANK_PER 4
#endif
    constexpr int kPlacePer = PIN_PLACE_PER;
    const int nplace = (int)((n + kPlacePer * kPartThreads - 1) / (kPlacePer * kPartThreads));
    auto launch = [&](auto per_tag, auto maxt_tag) {
        constexpr int PER = decltype(per_tag)::value;
        constexpr int MAXT = decltype(maxt_tag)::value;
        const int nblk = (int)((n + PER * kPartThreads - 1) / (PER * kPartThreads));
        hipLaunchKernelGGL((k_tile_rank<PER, MAXT>), dim3(nblk), dim3(kPartThreads), 0, s, q, n, t, tot, tk);
        hipLaunchKernelGGL((k_tile_place<kPlacePer, MAXT>), dim3(nplace), dim3(kPartThreads), 0, s, q, n, t.ntiles, tot,
                           done, tk, q4, order);
    };
    if (n <= (1 << 19)) launch(std::integral_constant<int, PIN_RANK_PER>(), std::integral_constant<int, kMaxTiles>());
    else if (!large) launch(std::integral_constant<int, 16>(), std::integral_constant<int, kMaxTiles>());
    else launch(std::integral_constant<int, 16>(), std::integral_constant<int, kMaxTilesLarge>());
    return hipGetLastError() == hipSuccess ? PIN_OK : PIN_ERR_HIP;
}

// The stable tile sort (pin_query_sort_stable): tile keys, a rocPRIM radix sort of (key, index)
// pairs over the key bits -- LSD radix sorting is stable, so a tile keeps its queries in input
// order -- then the placement.  Same tile map as sort_queries.
constexpr int kStableKeyBits = 14;
static_assert((1 << kStableKeyBits) >= kMaxTilesLarge && (1 << kStableKeyBits) >= kMaxTiles, "tile key bits");

__global__ void __launch_bounds__(kBlock)
k_tile_keys(const float* __restrict__ q, int64_t n, TileMap t, unsigned* __restrict__ keys,
            unsigned* __restrict__ vals) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    keys[i] = (unsigned)tile_of(q[3 * i], q[3 * i + 1], q[3 * i + 2], t);
    vals[i] = (unsigned)i;
}

__global__ void __launch_bounds__(kBlock)
k_tile_place_stable(const float* __restrict__ q, int64_t n, const unsigned* __restrict__ vals,
                    float4* __restrict__ q4, int* __restrict__ order) {
    const int64_t pos = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (pos >= n) return;
    const int64_t i = vals[pos];
    if (q4) q4[pos] = make_float4(q[3 * i], q[3 * i + 1], q[3 * i + 2], __int_as_float((int)i));
    if (order) order[pos] = (int)i;
}

struct StableSortWs {
    unsigned *k_in, *k_out, *v_in, *v_out;
    void* temp;
    size_t temp_bytes;
};

size_t stable_sort_temp_bytes(int64_t n) {
    size_t bytes = 0;
    if (rocprim::radix_sort_pairs(nullptr, bytes, (unsigned*)nullptr, (unsigned*)nullptr, (unsigned*)nullptr,
                                  (unsigned*)nullptr, (size_t)std::max<int64_t>(n, 1), 0, kStableKeyBits,
                                  (hipStream_t)0) != hipSuccess)
        return 0;
    return bytes;
}

inline int64_t align256(int64_t b) { return (b + 255) & ~(int64_t)255; }

StableSortWs stable_sort_ws(void* ws, int64_t n) {
    char* p = (char*)ws;
    const int64_t a = align256(4 * std::max<int64_t>(n, 1));
    StableSortWs w;
    w.k_in = (unsigned*)p;
    w.k_out = (unsigned*)(p + a);
    w.v_in = (unsigned*)(p + 2 * a);
    w.v_out = (unsigned*)(p + 3 * a);
    w.temp = p + 4 * a;
    w.temp_bytes = stable_sort_temp_bytes(n);
    return w;
}

// ------------------------------------------------------------------ drop-in query_feature
template <bool WF, bool PGO, class Src>
__device__ __forceinline__ void query_feature_body(const Src& src, const PinPoints& p, const float* __restrict__ q,
                                                   int64_t i, int nn_k, float* __restrict__ feat,
                                                   float* __restrict__ weights, int64_t* __restrict__ nn_counts,
                                                   float* __restrict__ cert_out, int* __restrict__ ids,
                                                   int* __restrict__ gids) {
    const int64_t iq = i >= 0 ? i : 0;   // i < 0: no query (the lane only completes its wave)
    const float qx = q[3 * iq], qy = q[3 * iq + 1], qz = q[3 * iq + 2];
    TopK tk;
    tk.init();
    const int nn = src.template scan<Src::kChunk>(qx, qy, qz, tk);
    resolve_ties(src, qx, qy, qz, nn_k, nn, tk, kTieAll);   // the reference's neighbour order (layout)
    Neighbours nb;
    load_topk(src, p, tk, nn, nn_k, qx, qy, qz, nb);
    const float cert = (cert_out && p.certainties) ? gather_certainty(src, nb) : 0.f;
    float x[kD];
#pragma unroll
    for (int d = 0; d < kD; ++d) x[d] = 0.f;
#pragma unroll
    for (int half = 0; half < kK / 4; ++half) {
        float xk[4][kD];
        float4 qt[4];
        if (half == 0) gather_inputs<PGO, 0, 4>(src, p, nb, xk, qt);
        else gather_inputs<PGO, 4, 4>(src, p, nb, xk, qt);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int j = half * 4 + t;
            if (j >= nn_k) break;
            if (WF) {
#pragma unroll
                for (int d = 0; d < kD; ++d) x[d] = x[d] + xk[t][d] * nb.w[j];
            } else {
                float* o = feat + (i * nn_k + j) * kD;
#pragma unroll
                for (int d = 0; d < kD; ++d) o[d] = xk[t][d];
            }
        }
    }
    if (WF) {
#pragma unroll
        for (int d = 0; d < kD; ++d) feat[i * kD + d] = x[d];
    }
#pragma unroll
    for (int j = 0; j < kK; ++j) {
        if (j >= nn_k) break;
        weights[i * nn_k + j] = nb.w[j];
        if (ids) ids[i * nn_k + j] = nb.id[j];
        if (gids) gids[i * nn_k + j] = nb.id[j] >= 0 ? src.gid(tk.g[j]) : -1;
    }
    if (nn_counts) nn_counts[i] = nn;
    if (cert_out) cert_out[i] = cert;
}

template <bool WF, bool PGO>
__global__ void __launch_bounds__(kBlock)
k_query_feature_fwd(const PinHash h, const PinPoints p, const float* __restrict__ q, int64_t n, int nn_k,
                    float* __restrict__ feat, float* __restrict__ weights, int64_t* __restrict__ nn_counts,
                    float* __restrict__ cert_out, int* __restrict__ ids, int* __restrict__ gids) {
    const int64_t i0 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if ((i0 & ~(int64_t)63) >= n) return;   // whole waves (resolve_ties): lanes past n redo query n-1
    const int64_t i = i0 < n ? i0 : n - 1;   // (identical values to the same addresses)
    const HashSource src(h, p);
    query_feature_body<WF, PGO>(src, p, q, i, nn_k, feat, weights, nn_counts, cert_out, ids, gids);
}

template <bool WF, bool PGO>
__global__ void __launch_bounds__(kBlock)
k_query_feature_fwd_grid(const PinGrid g, const PinPoints p, const float* __restrict__ q, int64_t n, int nn_k,
                         float* __restrict__ feat, float* __restrict__ weights, int64_t* __restrict__ nn_counts,
                         float* __restrict__ cert_out, int* __restrict__ ids, int* __restrict__ gids) {
    const int64_t i0 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if ((i0 & ~(int64_t)63) >= n) return;   // whole waves (resolve_ties): lanes past n redo query n-1
    const int64_t i = i0 < n ? i0 : n - 1;   // (identical values to the same addresses)
    const GridSource<false> src(g, p);
    query_feature_body<WF, PGO>(src, p, q, i, nn_k, feat, weights, nn_counts, cert_out, ids, gids);
}

// One 8-float row per lane added into dst[id * 8 ..] (id < 0: nothing), staged through the wave's
// LDS slice s (64 x 8 floats + 64 ids) and issued as 8 lanes x 32 contiguous bytes per atomic
// instruction -- the cheapest float-atomic shape measured (the training scatter's); one lane per
// row with 8 separate 4-B atomics hits 64 lines per instruction.  Every lane of the wave calls this.
__device__ __forceinline__ void wave_rows_atomic(float* s, int id, const float (&g)[kF], float* __restrict__ dst) {
    const int lane = threadIdx.x & 63;
    int* sid = (int*)(s + 64 * kF);
    wave_lds_sync();   // the previous call's readers are done
#pragma unroll
    for (int d = 0; d < kF; ++d) s[lane * kF + d] = g[d];
    sid[lane] = id;
    wave_lds_sync();
#pragma unroll
    for (int u = 0; u < kF; ++u) {
        const int e = u * 64 + lane;
        const int rid = sid[e >> 3];
        if (rid >= 0) atomicAdd(dst + (int64_t)rid * kF + (e & (kF - 1)), s[e]);
    }
}

template <bool WF, bool PGO>
__global__ void __launch_bounds__(kBlock)
k_query_feature_bwd(const PinPoints p, const float* __restrict__ q, int64_t n, int nn_k, const int* __restrict__ ids,
                    const int* __restrict__ gids, const float* __restrict__ weights,
                    const float* __restrict__ gfeat, const float* __restrict__ gw, float* __restrict__ gq_out,
                    float* __restrict__ gF) {
    __shared__ float s_sc[kBlock / 64][64 * kF + 64];
    const int64_t i0 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if ((i0 & ~(int64_t)63) >= n) return;   // whole waves past the end (the scatter is wave-wide)
    const bool live = i0 < n;
    const int64_t i = live ? i0 : 0;          // dead lanes compute row 0 and write nothing
    const float qx = q[3 * i], qy = q[3 * i + 1], qz = q[3 * i + 2];
    const float4* __restrict__ rec = (const float4*)p.records;
    float gx[kD];
    if (WF) {
#pragma unroll
        for (int d = 0; d < kD; ++d) gx[d] = gfeat ? gfeat[i * kD + d] : 0.f;
    }
    float u[kK], w[kK], dw[kK], pg[kK][3];
    int id[kK];
    float S = 0.f;
    float gq[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < kK; ++j) {
        id[j] = -1;
        u[j] = 0.f;
        w[j] = 0.f;
        dw[j] = 0.f;
        pg[j][0] = pg[j][1] = pg[j][2] = 0.f;
        if (j >= nn_k) continue;
        const int g = live ? gids[i * nn_k + j] : -1;
        if (g < 0) continue;
        id[j] = ids[i * nn_k + j];
        const float4 r = rec[g];
        const float d2 = dist2(r.x, r.y, r.z, qx, qy, qz);
        u[j] = 1.0f / (d2 + kIdwEps);
        S = S + u[j];
        w[j] = weights[i * nn_k + j];
        pg[j][0] = qx - r.x;
        pg[j][1] = qy - r.y;
        pg[j][2] = qz - r.z;
        float v[3];
        float px = r.x, py = r.y, pz = r.z;
        if (__float_as_int(r.w) & PIN_RECORD_UNFAITHFUL) {
            px = p.positions[3 * (int64_t)id[j]];
            py = p.positions[3 * (int64_t)id[j] + 1];
            pz = p.positions[3 * (int64_t)id[j] + 2];
        }
        v[0] = qx - px;
        v[1] = qy - py;
        v[2] = qz - pz;
        float4 qt = make_float4(1.f, 0.f, 0.f, 0.f);
        if (PGO) {
            qt = ((const float4*)p.orientations)[id[j]];
            quat_rotate_passive(qt, v[0], v[1], v[2]);
        }
        // dL/dw_j and the direct gradients through feature and vector
        float gvec[3];
        float gfe[kF];
        if (WF) {
            const float4* fr = (const float4*)(p.features + (int64_t)id[j] * kF);
            const float4 f0 = fr[0], f1 = fr[1];
            const float f[kF] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
            float s = 0.f;
#pragma unroll
            for (int d = 0; d < kF; ++d) s = fmaf(gx[d], f[d], s);
#pragma unroll
            for (int d = 0; d < 3; ++d) s = fmaf(gx[kF + d], v[d], s);
            dw[j] = s;
#pragma unroll
            for (int d = 0; d < kF; ++d) gfe[d] = w[j] * gx[d];
#pragma unroll
            for (int d = 0; d < 3; ++d) gvec[d] = w[j] * gx[kF + d];
        } else {
            const float* G = gfeat ? gfeat + (i * nn_k + j) * kD : nullptr;
#pragma unroll
            for (int d = 0; d < kF; ++d) gfe[d] = G ? G[d] : 0.f;
#pragma unroll
            for (int d = 0; d < 3; ++d) gvec[d] = G ? G[kF + d] : 0.f;
        }
        if (gw) dw[j] += gw[i * nn_k + j];
        float r0 = gvec[0], r1 = gvec[1], r2 = gvec[2];
        if (PGO) quat_rotate_active(qt, gvec[0], gvec[1], gvec[2], r0, r1, r2);
        gq[0] += r0;
        gq[1] += r1;
        gq[2] += r2;
    }
    if (gF) {   // the feature rows: w_j G[0:8] (weighted_first) or G_j[0:8], wave-staged
        for (int j = 0; j < nn_k; ++j) {
            float gfe[kF];
            const bool ok = id[j] >= 0;
            if (WF) {
#pragma unroll
                for (int d = 0; d < kF; ++d) gfe[d] = w[j] * gx[d];
            } else {
                const float* G = (gfeat && ok) ? gfeat + (i * nn_k + j) * kD : nullptr;
#pragma unroll
                for (int d = 0; d < kF; ++d) gfe[d] = G ? G[d] : 0.f;
            }
            wave_rows_atomic(s_sc[threadIdx.x >> 6], ok ? id[j] : -1, gfe, gF);
        }
    }
    if (!gq_out || !live) return;
    if (S > 0.f) {
        float wbar = 0.f;
#pragma unroll
        for (int j = 0; j < kK; ++j) wbar = fmaf(w[j], dw[j], wbar);
        const float invS = 1.f / S;
#pragma unroll
        for (int j = 0; j < kK; ++j) {
            if (id[j] < 0) continue;
            const float coef = -2.f * u[j] * u[j] * (dw[j] - wbar) * invS;
#pragma unroll
            for (int d = 0; d < 3; ++d) gq[d] = fmaf(coef, pg[j][d], gq[d]);
        }
    }
    gq_out[3 * i] = gq[0];
    gq_out[3 * i + 1] = gq[1];
    gq_out[3 * i + 2] = gq[2];
}

// Double backward of k_query_feature_bwd (second order: get_gradient(..., create_graph=True),
// utils/tools.py:174-184, then a loss on the gradient).  With r_j = q - p_j (record position), u_j =
// 1/(|r_j|^2 + eps), S = sum u, w_j = u_j / S, x_j = [f_j, P_j (q - p~_j)] (P_j the passive PGO
// rotation), the first-order backward is
//   grad_q = sum_j P_j^T dx_j[8:11] + sum_j k_j (a_j - abar),  k_j = -2 u_j^2 r_j / S,
//   grad_f[id_j] += dx_j[0:8],
// with dx_j = w_j G, a_j = G . x_j + Gw_j (weighted_first; G = dL/dout [11]) or dx_j = G_j, a_j =
// Gw_j (per neighbour), abar = sum_j w_j a_j.  Given the upstream H_q = dL2/dgrad_q and H_f =
// dL2/dgrad_f, this returns dL2/dq, dL2/dG, dL2/dGw and (weighted_first) dL2/dfeatures in closed form:
//   h_j = H_q . k_j, H = sum h, e_j = h_j - H w_j = dL2/da_j = dL2/dGw_j
//   weighted_first: dL2/dG = sum_j (w_j [H_f[id_j], P_j H_q] + e_j x_j), dL2/df_j = e_j G[0:8]
//   per neighbour:  dL2/dG_j = [H_f[id_j], P_j H_q]
//   dL2/dq = sum_i du_i (s_i - sbar)/S + sum_i (a_i - abar) dh_i + sum_i e_i b_i - H sum_i du_i (a_i - abar)/S
//     du_i = -2 u_i^2 r_i, s_i = (P_i H_q) . G[8:11] + H_f[id_i] . G[0:8] (weighted_first, else 0),
//     b_i = P_i^T G[8:11] (weighted_first, else 0), sigma = sum du,
//     dh_i = -2/S (u_i^2 H_q - 4 u_i^3 (r_i . H_q) r_i) + 2 u_i^2 (r_i . H_q) sigma / S^2.
template <bool WF, bool PGO>
__global__ void __launch_bounds__(kBlock)
k_query_feature_bwd2(const PinPoints p, const float* __restrict__ q, int64_t n, int nn_k, const int* __restrict__ ids,
                     const int* __restrict__ gids, const float* __restrict__ weights,
                     const float* __restrict__ gfeat, const float* __restrict__ gw, const float* __restrict__ hq,
                     const float* __restrict__ hf, float* __restrict__ dq_out, float* __restrict__ dg_out,
                     float* __restrict__ dgw_out, float* __restrict__ dF) {
    __shared__ float s_sc[kBlock / 64][64 * kF + 64];
    const int64_t i0 = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if ((i0 & ~(int64_t)63) >= n) return;   // whole waves past the end (the scatter is wave-wide)
    const bool live = i0 < n;
    const int64_t i = live ? i0 : 0;          // dead lanes compute row 0 and write nothing
    const float qx = q[3 * i], qy = q[3 * i + 1], qz = q[3 * i + 2];
    const float4* __restrict__ rec = (const float4*)p.records;
    const float H3[3] = {hq ? hq[3 * i] : 0.f, hq ? hq[3 * i + 1] : 0.f, hq ? hq[3 * i + 2] : 0.f};
    float G[kD];
#pragma unroll
    for (int d = 0; d < kD; ++d) G[d] = (WF && gfeat) ? gfeat[i * kD + d] : 0.f;
    float u[kK], w[kK], a[kK], sj[kK], r[kK][3], ph[kK][3], b[kK][3];
    int id[kK];
    float S = 0.f;
#pragma unroll
    for (int j = 0; j < kK; ++j) {
        id[j] = -1;
        u[j] = w[j] = a[j] = sj[j] = 0.f;
#pragma unroll
        for (int d = 0; d < 3; ++d) r[j][d] = ph[j][d] = b[j][d] = 0.f;
        if (j >= nn_k) continue;
        const int g = live ? gids[i * nn_k + j] : -1;
        if (g < 0) continue;
        id[j] = ids[i * nn_k + j];
        const float4 rc = rec[g];
        u[j] = 1.0f / (dist2(rc.x, rc.y, rc.z, qx, qy, qz) + kIdwEps);
        S = S + u[j];
        w[j] = weights[i * nn_k + j];
        r[j][0] = qx - rc.x;
        r[j][1] = qy - rc.y;
        r[j][2] = qz - rc.z;
        float px = rc.x, py = rc.y, pz = rc.z;
        if (__float_as_int(rc.w) & PIN_RECORD_UNFAITHFUL) {
            px = p.positions[3 * (int64_t)id[j]];
            py = p.positions[3 * (int64_t)id[j] + 1];
            pz = p.positions[3 * (int64_t)id[j] + 2];
        }
        float v[3] = {qx - px, qy - py, qz - pz};
        float4 qt = make_float4(1.f, 0.f, 0.f, 0.f);
        ph[j][0] = H3[0]; ph[j][1] = H3[1]; ph[j][2] = H3[2];
        if (PGO) {
            qt = ((const float4*)p.orientations)[id[j]];
            quat_rotate_passive(qt, v[0], v[1], v[2]);
            quat_rotate_passive(qt, ph[j][0], ph[j][1], ph[j][2]);   // P_j H_q
        }
        float hfj[kF];
#pragma unroll
        for (int d = 0; d < kF; ++d) hfj[d] = hf ? hf[(int64_t)id[j] * kF + d] : 0.f;
        if (WF) {
            const float4* fr = (const float4*)(p.features + (int64_t)id[j] * kF);
            const float4 f0 = fr[0], f1 = fr[1];
            const float f[kF] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
            float s = 0.f, t = 0.f;
#pragma unroll
            for (int d = 0; d < kF; ++d) {
                s = fmaf(G[d], f[d], s);
                t = fmaf(hfj[d], G[d], t);
            }
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                s = fmaf(G[kF + d], v[d], s);
                t = fmaf(ph[j][d], G[kF + d], t);
            }
            a[j] = s;
            sj[j] = t;
            float b0 = G[kF], b1 = G[kF + 1], b2 = G[kF + 2];
            if (PGO) quat_rotate_active(qt, G[kF], G[kF + 1], G[kF + 2], b0, b1, b2);   // P_j^T G[8:11]
            b[j][0] = b0; b[j][1] = b1; b[j][2] = b2;
            // x_j is needed again for dL2/dG once e_j is known: re-read in the second pass (not kept live)
        } else {
            if (dg_out) {   // dL2/dG_j = [H_f[id_j], P_j H_q]
                float* o = dg_out + (i * nn_k + j) * kD;
#pragma unroll
                for (int d = 0; d < kF; ++d) o[d] = hfj[d];
#pragma unroll
                for (int d = 0; d < 3; ++d) o[kF + d] = ph[j][d];
            }
        }
        if (gw) a[j] += gw[i * nn_k + j];
    }
    if (!WF && dg_out && live) {   // invalid / padded neighbour slots get zeros
#pragma unroll
        for (int j = 0; j < kK; ++j) {
            if (j >= nn_k || id[j] >= 0) continue;
            float* o = dg_out + (i * nn_k + j) * kD;
#pragma unroll
            for (int d = 0; d < kD; ++d) o[d] = 0.f;
        }
    }
    const float invS = S > 0.f ? 1.f / S : 0.f;
    float h[kK], H = 0.f, abar = 0.f, sbar = 0.f, sig[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < kK; ++j) {
        const float c = -2.f * u[j] * u[j];                 // du_j = c r_j
        h[j] = c * invS * (H3[0] * r[j][0] + H3[1] * r[j][1] + H3[2] * r[j][2]);
        H += h[j];
        abar = fmaf(w[j], a[j], abar);
        sbar = fmaf(w[j], sj[j], sbar);
#pragma unroll
        for (int d = 0; d < 3; ++d) sig[d] = fmaf(c, r[j][d], sig[d]);
    }
    float dq[3] = {0.f, 0.f, 0.f};
    float dG[kD];
    float ej[kK];   // e_j, for the wave-staged dL2/df_j = e_j G[0:8] after the loop
#pragma unroll
    for (int d = 0; d < kD; ++d) dG[d] = 0.f;
#pragma unroll
    for (int j = 0; j < kK; ++j) {
        ej[j] = 0.f;
        if (id[j] < 0) continue;
        const float e = h[j] - H * w[j];
        ej[j] = e;
        if (dgw_out) dgw_out[i * nn_k + j] = e;
        const float c = -2.f * u[j] * u[j];
        const float rh = r[j][0] * H3[0] + r[j][1] * H3[1] + r[j][2] * H3[2];
        const float da = a[j] - abar;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const float du = c * r[j][d];
            // dPhi: du (s - sbar) / S;  -H du (a - abar) / S
            float t = du * ((sj[j] - sbar) - H * da) * invS;
            // (a - abar) dh_j
            const float dh = -2.f * invS * (u[j] * u[j] * H3[d] - 4.f * u[j] * u[j] * u[j] * rh * r[j][d]) +
                             2.f * u[j] * u[j] * rh * sig[d] * invS * invS;
            t = fmaf(da, dh, t);
            t = fmaf(e, b[j][d], t);
            dq[d] += t;
        }
        if (WF) {
            // x_j again (features and the rotated vector) for dL2/dG and dL2/df_j
            const int64_t ij = id[j];
            const float4* fr = (const float4*)(p.features + ij * kF);
            const float4 f0 = fr[0], f1 = fr[1];
            const float f[kF] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
            const int g = gids[i * nn_k + j];
            const float4 rc = rec[g];
            float px = rc.x, py = rc.y, pz = rc.z;
            if (__float_as_int(rc.w) & PIN_RECORD_UNFAITHFUL) {
                px = p.positions[3 * ij];
                py = p.positions[3 * ij + 1];
                pz = p.positions[3 * ij + 2];
            }
            float v[3] = {qx - px, qy - py, qz - pz};
            if (PGO) quat_rotate_passive(((const float4*)p.orientations)[ij], v[0], v[1], v[2]);
#pragma unroll
            for (int d = 0; d < kF; ++d) {
                const float hfd = hf ? hf[ij * kF + d] : 0.f;
                dG[d] = fmaf(w[j], hfd, fmaf(e, f[d], dG[d]));
            }
#pragma unroll
            for (int d = 0; d < 3; ++d) dG[kF + d] = fmaf(w[j], ph[j][d], fmaf(e, v[d], dG[kF + d]));
        }
    }
    if (WF && dF) {
        for (int j = 0; j < nn_k; ++j) {
            float gfe[kF];
#pragma unroll
            for (int d = 0; d < kF; ++d) gfe[d] = ej[j] * G[d];
            wave_rows_atomic(s_sc[threadIdx.x >> 6], id[j], gfe, dF);
        }
    }
    if (!live) return;
    if (WF && dg_out) {
#pragma unroll
        for (int d = 0; d < kD; ++d) dg_out[i * kD + d] = dG[d];
    }
    if (dgw_out) {   // invalid / padded neighbour slots
#pragma unroll
        for (int j = 0; j < kK; ++j)
            if (j < nn_k && id[j] < 0) dgw_out[i * nn_k + j] = 0.f;
    }
    if (dq_out) {
        dq_out[3 * i] = dq[0];
        dq_out[3 * i + 1] = dq[1];
        dq_out[3 * i + 2] = dq[2];
    }
}

// ------------------------------------------------------------------ training side effects
__global__ void __launch_bounds__(kBlock)
k_train_scatter(const int* __restrict__ ids, const float* __restrict__ w, int64_t total, int nn_k,
                const int64_t* __restrict__ qts, float* __restrict__ cert, int64_t* __restrict__ ts) {
    const int64_t e = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (e >= total) return;
    const int id = ids[e];
    if (id < 0) return;
    if (cert) atomicAdd(cert + id, w[e]);
    if (qts && ts) atomicMax((unsigned long long*)(ts + id), (unsigned long long)qts[e / nn_k]);
}

}  // namespace

// ===================================================================== C ABI
extern "C" {

int pin_build_records(const float* positions, int64_t num_points, int32_t query_locally, const int64_t* global2local,
                      const int64_t* ts_create, const float* travel_dist, int64_t travel_len, int64_t cur_ts,
                      float diff_travel_dist_local, const float* local_positions, int64_t local_rows, float* records,
                      void* stream) {
    if (num_points < 0 || (num_points > 0 && (!positions || !records))) return PIN_ERR_ARG;
    if (query_locally && travel_dist && (!ts_create || cur_ts < 0 || cur_ts >= travel_len)) return PIN_ERR_ARG;
    if (num_points == 0) return PIN_OK;
    hipLaunchKernelGGL(k_build_records, grid_for(num_points), dim3(kBlock), 0, as_stream(stream), positions,
                       num_points, query_locally, global2local, ts_create, travel_dist, cur_ts, diff_travel_dist_local,
                       local_positions, local_rows, (float4*)records);
    return launch_status();
}

int pin_neighbor_cells(const int32_t* host_dx, int32_t num_cells, int64_t buffer_size, int32_t* cells_out,
                       void* stream) {
    if (!host_dx || !cells_out || num_cells <= 0 || buffer_size <= 0 || buffer_size >= (1ll << 31)) return PIN_ERR_ARG;
    std::vector<int32_t> cells((size_t)pin_cells_padded(num_cells), 0);
    for (int c = 0; c < num_cells; ++c) {
        const int64_t dx = host_dx[3 * c], dy = host_dx[3 * c + 1], dz = host_dx[3 * c + 2];
        int64_t r = (dx * kP0 + dy * kP1 + dz * kP2) % buffer_size;
        if (r < 0) r += buffer_size;
        cells[c] = (int32_t)r;
    }
    // pageable source: the copy is staged before the call returns
    if (hipMemcpyAsync(cells_out, cells.data(), cells.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                       as_stream(stream)) != hipSuccess)
        return PIN_ERR_HIP;
    return PIN_OK;
}

int pin_hash_rebuild(const float* positions, int64_t n, float resolution, int32_t* table, int64_t buffer_size,
                     void* stream) {
    if (n < 0 || !table || buffer_size <= 0 || buffer_size >= (1ll << 31) || resolution <= 0.f) return PIN_ERR_ARG;
    if (n > (int64_t)INT32_MAX) return PIN_ERR_UNSUPPORTED;
    if (n == 0) return PIN_OK;
    if (!positions) return PIN_ERR_ARG;
    hipLaunchKernelGGL(k_hash_rebuild, grid_for(n), dim3(kBlock), 0, as_stream(stream), positions, n, resolution,
                       table, buffer_size);
    return launch_status();
}

int pin_radius_search(const PinHash* hash, const PinPoints* pts, const float* q, int64_t n, float* dist2_out,
                      int64_t* idx_out, void* stream) {
    if (!hash_ok(hash) || !points_ok(pts) || n < 0 || (n > 0 && (!q || !dist2_out || !idx_out))) return PIN_ERR_ARG;
    if (n == 0) return PIN_OK;
    hipLaunchKernelGGL(k_radius_search, grid_for(n), dim3(kBlock), 0, as_stream(stream), *hash,
                       (const float4*)pts->records, q, n, dist2_out, idx_out);
    return launch_status();
}

int pin_query_certainty(const PinHash* hash, const PinPoints* pts, const float* q, int64_t n, float* certainty_out,
                        void* stream) {
    if (!hash_ok(hash) || !points_ok(pts) || !pts->certainties || n < 0 || (n > 0 && (!q || !certainty_out)))
        return PIN_ERR_ARG;
    if (n == 0) return PIN_OK;
    hipLaunchKernelGGL(k_query_certainty, grid_for(n), dim3(kBlock), 0, as_stream(stream), *hash,
                       (const float4*)pts->records, pts->certainties, q, n, certainty_out);
    return launch_status();
}

int pin_query_sdf(const PinHash* hash, const PinPoints* pts, const PinMlp* mlp, const float* q, int64_t n,
                  int32_t nn_k, int32_t weighted_first, int32_t zero_empty, float* sdf, float* grad, int32_t* nn_count,
                  float* certainty, float* sdf_std, void* stream) {
    if (!hash_ok(hash) || !points_ok(pts) || !mlp || !mlp->W1 || !mlp->b1 || !mlp->W2 || !mlp->b2 || n < 0)
        return PIN_ERR_ARG;
    if (!pts->features || !pts->certainties || (pts->after_pgo && !pts->orientations)) return PIN_ERR_ARG;
    if (nn_k < 1 || nn_k > kK) return PIN_ERR_UNSUPPORTED;
    if (n == 0) return PIN_OK;
    if (!q) return PIN_ERR_ARG;
    const bool g = grad != nullptr;
    const bool pgo = pts->after_pgo != 0;
    auto s = as_stream(stream);
    const bool mf = mlp->packed != nullptr && g;   // as query_sdf_grid
#define PIN_LAUNCH_SDF(WF, PGO, GRAD)                                                                              \
    do {                                                                                                          \
        if (mf && GRAD)                                                                                           \
            hipLaunchKernelGGL((k_query_sdf<WF, PGO, GRAD, GRAD>), grid_for(n), dim3(kBlock), 0, s, *hash, *pts,    \
                               *mlp, q, n, nn_k, zero_empty, sdf, grad, nn_count, certainty, sdf_std);              \
        else                                                                                                      \
            hipLaunchKernelGGL((k_query_sdf<WF, PGO, GRAD, false>), grid_for(n), dim3(kBlock), 0, s, *hash, *pts,   \
                               *mlp, q, n, nn_k, zero_empty, sdf, grad, nn_count, certainty, sdf_std);              \
    } while (0)
    if (weighted_first) {
        if (pgo) { if (g) PIN_LAUNCH_SDF(true, true, true); else PIN_LAUNCH_SDF(true, true, false); }
        else { if (g) PIN_LAUNCH_SDF(true, false, true); else PIN_LAUNCH_SDF(true, false, false); }
    } else {
        if (pgo) { if (g) PIN_LAUNCH_SDF(false, true, true); else PIN_LAUNCH_SDF(false, true, false); }
        else { if (g) PIN_LAUNCH_SDF(false, false, true); else PIN_LAUNCH_SDF(false, false, false); }
    }
#undef PIN_LAUNCH_SDF
    return launch_status();
}

int pin_query_feature_fwd(const PinHash* hash, const PinPoints* pts, const float* q, int64_t n, int32_t nn_k,
                          int32_t weighted_first, float* feat, float* weights, int64_t* nn_counts, float* certainty,
                          int32_t* ids, int32_t* gids, void* stream) {
    if (!hash_ok(hash) || !points_ok(pts) || !pts->features || n < 0) return PIN_ERR_ARG;
    if (pts->after_pgo && !pts->orientations) return PIN_ERR_ARG;
    if (nn_k < 1 || nn_k > kK) return PIN_ERR_UNSUPPORTED;
    if (n == 0) return PIN_OK;
    if (!q || !feat || !weights) return PIN_ERR_ARG;
    auto s = as_stream(stream);
    const bool pgo = pts->after_pgo != 0;
#define PIN_LAUNCH_FWD(WF, PGO)                                                                          \
    hipLaunchKernelGGL((k_query_feature_fwd<WF, PGO>), grid_for(n), dim3(kBlock), 0, s, *hash, *pts, q, n, \
                       nn_k, feat, weights, nn_counts, certainty, ids, gids)
    if (weighted_first) { if (pgo) PIN_LAUNCH_FWD(true, true); else PIN_LAUNCH_FWD(true, false); }
    else { if (pgo) PIN_LAUNCH_FWD(false, true); else PIN_LAUNCH_FWD(false, false); }
#undef PIN_LAUNCH_FWD
    return launch_status();
}

int pin_query_feature_bwd2(const PinPoints* pts, const float* q, int64_t n, int32_t nn_k, int32_t weighted_first,
                           const int32_t* ids, const int32_t* gids, const float* weights, const float* grad_feat,
                           const float* grad_weights, const float* up_q, const float* up_features, float* d_q,
                           float* d_grad_feat, float* d_grad_weights, float* d_features, void* stream) {
    if (!points_ok(pts) || !pts->features || n < 0) return PIN_ERR_ARG;
    if (pts->after_pgo && !pts->orientations) return PIN_ERR_ARG;
    if (nn_k < 1 || nn_k > kK) return PIN_ERR_UNSUPPORTED;
    if (n == 0) return PIN_OK;
    if (!q || !ids || !gids || !weights) return PIN_ERR_ARG;
    auto s = as_stream(stream);
    const bool pgo = pts->after_pgo != 0;
#define PIN_LAUNCH_BWD2(WF, PGO)                                                                                 \
    hipLaunchKernelGGL((k_query_feature_bwd2<WF, PGO>), grid_for(n), dim3(kBlock), 0, s, *pts, q, n, nn_k, ids, \
                       gids, weights, grad_feat, grad_weights, up_q, up_features, d_q, d_grad_feat,            \
                       d_grad_weights, weighted_first ? d_features : nullptr)
    if (weighted_first) { if (pgo) PIN_LAUNCH_BWD2(true, true); else PIN_LAUNCH_BWD2(true, false); }
    else { if (pgo) PIN_LAUNCH_BWD2(false, true); else PIN_LAUNCH_BWD2(false, false); }
#undef PIN_LAUNCH_BWD2
    return launch_status();
}

int pin_query_feature_bwd(const PinPoints* pts, const float* q, int64_t n, int32_t nn_k, int32_t weighted_first,
                          const int32_t* ids, const int32_t* gids, const float* weights, const float* grad_feat,
                          const float* grad_weights, float* grad_q, float* grad_features, void* stream) {
    if (!points_ok(pts) || !pts->features || n < 0) return PIN_ERR_ARG;
    if (pts->after_pgo && !pts->orientations) return PIN_ERR_ARG;
    if (nn_k < 1 || nn_k > kK) return PIN_ERR_UNSUPPORTED;
    if (n == 0) return PIN_OK;
    if (!q || !ids || !gids || !weights) return PIN_ERR_ARG;
    auto s = as_stream(stream);
    const bool pgo = pts->after_pgo != 0;
#define PIN_LAUNCH_BWD(WF, PGO)                                                                                \
    hipLaunchKernelGGL((k_query_feature_bwd<WF, PGO>), grid_for(n), dim3(kBlock), 0, s, *pts, q, n, nn_k, ids, \
                       gids, weights, grad_feat, grad_weights, grad_q, grad_features)
    if (weighted_first) { if (pgo) PIN_LAUNCH_BWD(true, true); else PIN_LAUNCH_BWD(true, false); }
    else { if (pgo) PIN_LAUNCH_BWD(false, true); else PIN_LAUNCH_BWD(false, false); }
#undef PIN_LAUNCH_BWD
    return launch_status();
}

int pin_train_scatter(const int32_t* ids, const float* weights, int64_t n, int32_t nn_k, const int64_t* query_ts,
                      float* certainties, int64_t* ts_update, void* stream) {
    if (n < 0 || nn_k < 1) return PIN_ERR_ARG;
    if (n == 0) return PIN_OK;
    if (!ids || !weights) return PIN_ERR_ARG;
    const int64_t total = n * nn_k;
    hipLaunchKernelGGL(k_train_scatter, grid_for(total), dim3(kBlock), 0, as_stream(stream), ids, weights, total,
                       nn_k, query_ts, certainties, ts_update);
    return launch_status();
}

static bool grid_ok(const PinGrid* g) {
    return g && g->bricks && g->crec && g->cgid && g->offsets && g->num_cells > 0 && g->resolution > 0.f &&
           g->dims.nbx > 0 && g->dims.nby > 0 && g->dims.nbz > 0 && (!g->fat || (g->cfeat && g->ccert));
}

// ------------------------------------------------------------------ decoder pack (pin_mlp_pack)
__global__ void __launch_bounds__(256) k_mlp_pack(const PinMlp m, unsigned char* __restrict__ out) {
    mlp_pack_block(m, out);
}

// pin_ref_sort_rows: the tie resolution's wave-parallel std::sort (resolve_ties, pin_device.h) on
// given rows, whole permutation out -- the test hook that pins it to torch's CPU sort on rows the
// geometry rarely produces (the depth-limit heap sort, heavy ties).  One wave per row.
__global__ void __launch_bounds__(kBlock)
k_ref_sort_rows(const float* __restrict__ keys, int n, int64_t rows, int32_t* __restrict__ order) {
    const int64_t row = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
    if (row >= rows) return;   // whole waves: kBlock is a multiple of 64
    const int lane = threadIdx.x & 63;
    const float* kr = keys + row * n;
    WaveRow r;
    r.ka = lane < n ? kr[lane] : 0.f;
    r.ga = lane;
    r.kb = lane + 64 < n ? kr[lane + 64] : 0.f;
    r.gb = lane + 64;
    wave_introsort_loop(r, n);
    int ra, rb;
    wave_final_rank(r, n, ra, rb);
    if (lane < n) order[row * n + ra] = r.ga;
    if (lane + 64 < n) order[row * n + rb] = r.gb;
}

int pin_ref_sort_rows(const float* keys, int32_t n, int64_t rows, int32_t* order, void* stream) {
    if (n < 1 || n > kRefSortMax || rows < 0 || (rows > 0 && (!keys || !order))) return PIN_ERR_ARG;
    if (rows == 0) return PIN_OK;
    const int64_t waves_per_block = kBlock / 64;
    hipLaunchKernelGGL(k_ref_sort_rows, dim3((unsigned)((rows + waves_per_block - 1) / waves_per_block)), dim3(kBlock),
                       0, as_stream(stream), keys, n, rows, order);
    return hipGetLastError() == hipSuccess ? PIN_OK : PIN_ERR_HIP;
}

int pin_mlp_pack(const PinMlp* mlp, void* packed, void* stream) {
    if (!mlp || !mlp->W1 || !mlp->b1 || !mlp->W2 || !mlp->b2 || !packed || ((uintptr_t)packed & 15)) return PIN_ERR_ARG;
    hipLaunchKernelGGL(k_mlp_pack, dim3(1), dim3(256), 0, as_stream(stream), *mlp, (unsigned char*)packed);
    return launch_status();
}

int pin_query_order(const PinGrid* grid, const float* q, int64_t n, int32_t* order, void* workspace, void* stream) {
    if (!grid_ok(grid) || n < 0 || (n > 0 && (!q || !order || !workspace)) || n > INT32_MAX) return PIN_ERR_ARG;
    if (n == 0) return PIN_OK;
    return sort_queries(*grid, q, n, nullptr, (int*)order, workspace, as_stream(stream));
}

int pin_query_sort(const PinGrid* grid, const float* q, int64_t n, float* q4, int32_t* order, void* workspace,
                   void* stream) {
    if (!grid_ok(grid) || n < 0 || (n > 0 && (!q || !q4 || !workspace)) || n > INT32_MAX) return PIN_ERR_ARG;
    if (n == 0) return PIN_OK;
    return sort_queries(*grid, q, n, (float4*)q4, (int*)order, workspace, as_stream(stream));
}


int64_t pin_query_sort_stable_workspace_bytes(int64_t n) {
    if (n < 0) return PIN_ERR_ARG;
    const size_t t = stable_sort_temp_bytes(n);
    if (t == 0) return PIN_ERR_HIP;
    return 4 * align256(4 * std::max<int64_t>(n, 1)) + (int64_t)t;
}

int pin_query_sort_stable(const PinGrid* grid, const float* q, int64_t n, float* q4, int32_t* order, void* workspace,
                          void* stream) {
    if (!grid_ok(grid) || n < 0 || (n > 0 && (!q || (!q4 && !order) || !workspace)) || n > INT32_MAX)
        return PIN_ERR_ARG;
    if (n == 0) return PIN_OK;
    auto s = as_stream(stream);
    const TileMap t = tile_map(*grid, n >= kLargeBatch ? kMaxTilesLarge : kMaxTiles);
    StableSortWs w = stable_sort_ws(workspace, n);
    if (w.temp_bytes == 0) return PIN_ERR_HIP;
    hipLaunchKernelGGL(k_tile_keys, grid_for(n), dim3(kBlock), 0, s, q, n, t, w.k_in, w.v_in);
    size_t tb = w.temp_bytes;
    if (rocprim::radix_sort_pairs(w.temp, tb, w.k_in, w.k_out, w.v_in, w.v_out, (size_t)n, 0, kStableKeyBits, s) !=
        hipSuccess)
        return PIN_ERR_HIP;
    hipLaunchKernelGGL(k_tile_place_stable, grid_for(n), dim3(kBlock), 0, s, q, n, w.v_out, (float4*)q4, (int*)order);
    return launch_status();
}

// argument checks of the grid SDF query, before anything is launched (the tiled entry sorts first)
static int query_sdf_grid_args(const PinGrid* grid, const PinPoints* pts, const PinMlp* mlp, int64_t n,
                               int32_t nn_k) {
    if (!grid_ok(grid) || !points_ok(pts) || !mlp || !mlp->W1 || !mlp->b1 || !mlp->W2 || !mlp->b2 || n < 0)
        return PIN_ERR_ARG;
    const bool fat = grid->fat != 0;
    if ((!fat && (!pts->features || !pts->certainties)) || (pts->after_pgo && !pts->orientations))
        return PIN_ERR_ARG;
    if (nn_k < 1 || nn_k > kK) return PIN_ERR_UNSUPPORTED;
    if (n > INT32_MAX) return PIN_ERR_ARG;
    return PIN_OK;
}

static int query_sdf_grid(const PinGrid* grid, const PinPoints* pts, const PinMlp* mlp, const float* q,
                          const float* q4, int64_t n, int32_t nn_k, int32_t weighted_first, int32_t zero_empty,
                          float* sdf, float* grad, int32_t* nn_count, float* certainty, float* sdf_std,
                          const int32_t* order, void* stream, int out_slot = 0) {
    const int rc = query_sdf_grid_args(grid, pts, mlp, n, nn_k);
    if (rc != PIN_OK) return rc;
    if (n == 0) return PIN_OK;
    if (!q && !q4) return PIN_ERR_ARG;
    if (out_slot && !q4) return PIN_ERR_ARG;   // tile-order outputs are read against q4
    const bool fat = grid->fat != 0;
    const bool g = grad != nullptr;
    const bool pgo = pts->after_pgo != 0;
    // the matrix-core decoder pays off where the decoder carries the input gradient (262K queries:
    // 54.8 -> 47.8 us weighted_first, 97 -> 69 us per-neighbour); SDF-only decodes measured even
    // (45 / 91 us) and stay on the VALU
    const bool mf = mlp->packed != nullptr && g;
    auto s = as_stream(stream);
#define PIN_LAUNCH_SDFG(WF, PGO, GRAD, FAT, MF)                                                                   \
    hipLaunchKernelGGL((k_query_sdf_grid<WF, PGO, GRAD, FAT, MF>), grid_for(n), dim3(kBlock), 0, s, *grid, *pts, \
                       *mlp, q, (const float4*)q4, n, nn_k, zero_empty, sdf, grad, nn_count, certainty, sdf_std,   \
                       (const int*)order, out_slot)
#define PIN_SDFG_MF(WF, PGO, GRAD, FAT) \
    do { if (mf && GRAD) PIN_LAUNCH_SDFG(WF, PGO, GRAD, FAT, GRAD); else PIN_LAUNCH_SDFG(WF, PGO, GRAD, FAT, false); } while (0)
#define PIN_SDFG_FAT(WF, PGO, GRAD) \
    do { if (fat) PIN_SDFG_MF(WF, PGO, GRAD, true); else PIN_SDFG_MF(WF, PGO, GRAD, false); } while (0)
    if (weighted_first) {
        if (pgo) { if (g) PIN_SDFG_FAT(true, true, true); else PIN_SDFG_FAT(true, true, false); }
        else { if (g) PIN_SDFG_FAT(true, false, true); else PIN_SDFG_FAT(true, false, false); }
    } else {
        if (pgo) { if (g) PIN_SDFG_FAT(false, true, true); else PIN_SDFG_FAT(false, true, false); }
        else { if (g) PIN_SDFG_FAT(false, false, true); else PIN_SDFG_FAT(false, false, false); }
    }
#undef PIN_SDFG_FAT
#undef PIN_SDFG_MF
#undef PIN_LAUNCH_SDFG
    return launch_status();
}

int pin_query_sdf_grid_sorted_ex(const PinGrid* grid, const PinPoints* pts, const PinMlp* mlp, const float* q4,
                                 int64_t n, int32_t nn_k, int32_t weighted_first, int32_t zero_empty, float* sdf,
                                 float* grad, int32_t* nn_count, float* certainty, float* sdf_std, int32_t flags,
                                 void* stream) {
    if ((n > 0 && !q4) || (flags & ~PIN_QUERY_OUT_TILE)) return PIN_ERR_ARG;
    return query_sdf_grid(grid, pts, mlp, nullptr, q4, n, nn_k, weighted_first, zero_empty, sdf, grad, nn_count,
                          certainty, sdf_std, nullptr, stream, (flags & PIN_QUERY_OUT_TILE) ? 1 : 0);
}

int pin_query_sdf_grid_sorted(const PinGrid* grid, const PinPoints* pts, const PinMlp* mlp, const float* q4,
                              int64_t n, int32_t nn_k, int32_t weighted_first, int32_t zero_empty, float* sdf,
                              float* grad, int32_t* nn_count, float* certainty, float* sdf_std, void* stream) {
    return pin_query_sdf_grid_sorted_ex(grid, pts, mlp, q4, n, nn_k, weighted_first, zero_empty, sdf, grad, nn_count,
                                        certainty, sdf_std, 0, stream);
}

int pin_query_sdf_grid_tiled_ex(const PinGrid* grid, const PinPoints* pts, const PinMlp* mlp, const float* q,
                                int64_t n, int32_t nn_k, int32_t weighted_first, int32_t zero_empty, float* sdf,
                                float* grad, int32_t* nn_count, float* certainty, float* sdf_std, float* q4,
                                void* workspace, int32_t flags, void* stream) {
    if (n < 0 || (n > 0 && (!q || !q4 || !workspace)) || (flags & ~PIN_QUERY_OUT_TILE)) return PIN_ERR_ARG;
    const int rc = query_sdf_grid_args(grid, pts, mlp, n, nn_k);   // every check before the sort launches
    if (rc != PIN_OK) return rc;
    if (n == 0) return PIN_OK;
    // the three launches leave the host back to back: the query kernel is queued before the
    // sort has finished, so the GPU does not wait for the host between them
    const int rs = sort_queries(*grid, q, n, (float4*)q4, nullptr, workspace, as_stream(stream));
    if (rs != PIN_OK) return rs;
    return query_sdf_grid(grid, pts, mlp, nullptr, q4, n, nn_k, weighted_first, zero_empty, sdf, grad, nn_count,
                          certainty, sdf_std, nullptr, stream, (flags & PIN_QUERY_OUT_TILE) ? 1 : 0);
}

int pin_query_sdf_grid_tiled(const PinGrid* grid, const PinPoints* pts, const PinMlp* mlp, const float* q,
                             int64_t n, int32_t nn_k, int32_t weighted_first, int32_t zero_empty, float* sdf,
                             float* grad, int32_t* nn_count, float* certainty, float* sdf_std, float* q4,
                             void* workspace, void* stream) {
    return pin_query_sdf_grid_tiled_ex(grid, pts, mlp, q, n, nn_k, weighted_first, zero_empty, sdf, grad, nn_count,
                                       certainty, sdf_std, q4, workspace, 0, stream);
}

int pin_query_sdf_grid(const PinGrid* grid, const PinPoints* pts, const PinMlp* mlp, const float* q, int64_t n,
                       int32_t nn_k, int32_t weighted_first, int32_t zero_empty, float* sdf, float* grad,
                       int32_t* nn_count, float* certainty, float* sdf_std, const int32_t* order, void* stream) {
    if (n > 0 && !q) return PIN_ERR_ARG;
    return query_sdf_grid(grid, pts, mlp, q, nullptr, n, nn_k, weighted_first, zero_empty, sdf, grad, nn_count,
                          certainty, sdf_std, order, stream);
}

// One iteration of the tracking loop in one call (utils/tracker.py:92-159 body): pose the source
// cloud (or re-pose its tile-sorted rows), the fused SDF + gradient query, the normal equations,
// the device solve (T = dT T) and an asynchronous copy of accumulators + status + dT to the host.
int pin_reg_iteration(const PinGrid* grid, const PinHash* hash, const PinPoints* pts, const PinMlp* mlp,
                      const PinRegIter* it, int32_t first, const double* pose_in, double* pose_out, void* stream) {
    if (!it || !pts || !mlp || !pose_in || !pose_out || it->n < 0 || !it->reg_ws || !it->acc_status_dt) return PIN_ERR_ARG;
    if ((grid == nullptr) == (hash == nullptr)) return PIN_ERR_ARG;
    const int64_t n = it->n;
    const bool sorted = it->q4 != nullptr;
    if (sorted && (!grid || (first && !it->order_ws))) return PIN_ERR_ARG;
    if (n > 0 && (!it->src || !it->sdf || !it->grad || !it->nn_count || (!sorted && !it->cur))) return PIN_ERR_ARG;
    const int rc = grid ? query_sdf_grid_args(grid, pts, mlp, n, it->nn_k) : PIN_OK;
    if (rc != PIN_OK) return rc;
    auto s = as_stream(stream);
    float* std_out = it->weighted_first ? nullptr : it->sdf_std;
    int r = PIN_OK;
    if (n > 0) {
        if (sorted && first) {
            r = pin_transform_points(it->src, n, pose_in, it->cur, stream);
            if (r == PIN_OK) r = sort_queries(*grid, it->cur, n, (float4*)it->q4, nullptr, it->order_ws, s);
        } else if (sorted) {
            r = pin_transform_points_sorted(it->src, n, pose_in, it->q4, stream);
        } else {
            r = pin_transform_points(it->src, n, pose_in, it->cur, stream);
        }
        if (r != PIN_OK) return r;
        if (grid)
            r = query_sdf_grid(grid, pts, mlp, sorted ? nullptr : it->cur, sorted ? it->q4 : nullptr, n, it->nn_k,
                               it->weighted_first, 0, it->sdf, it->grad, it->nn_count, nullptr, std_out, nullptr, stream,
                               sorted ? 1 : 0);
        else
            r = pin_query_sdf(hash, pts, mlp, it->cur, n, it->nn_k, it->weighted_first, 0, it->sdf, it->grad,
                              it->nn_count, nullptr, std_out, stream);
        if (r != PIN_OK) return r;
    }
    PinRegParams prm = it->prm;
    prm.q4_points = sorted ? 1 : 0;
    double* acc = it->acc_status_dt;
    double* status = acc + PIN_REG_NACC;
    double* dT = status + PIN_REG_NSTATUS;
    r = pin_reg_step(sorted ? it->q4 : it->cur, it->sdf, it->grad, it->nn_count, std_out, it->labels, n, &prm,
                     it->reg_ws, acc, it->lm_lambda, pose_in, dT, pose_out, status, stream);
    if (r != PIN_OK) return r;
    if (it->host_out &&
        hipMemcpyAsync(it->host_out, acc, sizeof(double) * (PIN_REG_NACC + PIN_REG_NSTATUS + 16), hipMemcpyDeviceToHost,
                       s) != hipSuccess)
        return PIN_ERR_HIP;
    return PIN_OK;
}

int pin_query_feature_fwd_grid(const PinGrid* grid, const PinPoints* pts, const float* q, int64_t n, int32_t nn_k,
                               int32_t weighted_first, float* feat, float* weights, int64_t* nn_counts,
                               float* certainty, int32_t* ids, int32_t* gids, void* stream) {
    if (!grid_ok(grid) || !points_ok(pts) || !pts->features || n < 0) return PIN_ERR_ARG;
    if (pts->after_pgo && !pts->orientations) return PIN_ERR_ARG;
    if (nn_k < 1 || nn_k > kK) return PIN_ERR_UNSUPPORTED;
    if (n == 0) return PIN_OK;
    if (!q || !feat || !weights) return PIN_ERR_ARG;
    auto s = as_stream(stream);
    const bool pgo = pts->after_pgo != 0;
#define PIN_LAUNCH_FWDG(WF, PGO)                                                                                \
    hipLaunchKernelGGL((k_query_feature_fwd_grid<WF, PGO>), grid_for(n), dim3(kBlock), 0, s, *grid, *pts, q, n, \
                       nn_k, feat, weights, nn_counts, certainty, ids, gids)
    if (weighted_first) { if (pgo) PIN_LAUNCH_FWDG(true, true); else PIN_LAUNCH_FWDG(true, false); }
    else { if (pgo) PIN_LAUNCH_FWDG(false, true); else PIN_LAUNCH_FWDG(false, false); }
#undef PIN_LAUNCH_FWDG
    return launch_status();
}

}  // extern "C"
