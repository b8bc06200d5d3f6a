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

namespace pin {

constexpr int kF = PIN_FEATURE_DIM;      // feature_dim
constexpr int kD = kF + 3;               // decoder input: feature + neighbour vector
constexpr int kH = PIN_HIDDEN_DIM;       // geo_mlp_hidden_dim
constexpr int kK = PIN_MAX_NN_K;         // top-k capacity
constexpr int kBlock = 256;
constexpr int kIdMask = PIN_RECORD_UNFAITHFUL - 1;
constexpr int64_t kP0 = 73856093LL, kP1 = 19349669LL, kP2 = 83492791LL;  // neural_points.py:69
constexpr float kInvalidDist2 = 9e3f;    // neural_points.py:561
constexpr float kIdwEps = 1e-15f;        // neural_points.py:618

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

// Sorted (ascending) register list of the k nearest candidates.  Ties keep candidate
// order (cell order), matching the stable sort of the CPU reference (:561-565).
struct TopK {
    float d[kK];
    int g[kK];
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int j = 0; j < kK; ++j) { d[j] = kInvalidDist2; g[j] = -1; }
    }
    __device__ __forceinline__ void insert(float x, int gi) {
        bool c[kK];
#pragma unroll
        for (int j = 0; j < kK; ++j) c[j] = d[j] <= x;
#pragma unroll
        for (int j = kK - 1; j > 0; --j) {
            const float nd = c[j] ? d[j] : (c[j - 1] ? x : d[j - 1]);
            const int ng = c[j] ? g[j] : (c[j - 1] ? gi : g[j - 1]);
            d[j] = nd;
            g[j] = ng;
        }
        if (!c[0]) { d[0] = x; g[0] = gi; }
    }
};

// Probe every neighbour cell of q, reject empty / filtered / too-far candidates and keep
// the k nearest (neural_points.py:459-509, :555-565).  Returns nn_count (valid candidates
// before truncation, :557).  CH table probes are issued before their records are read.
template <int CH>
__device__ __forceinline__ int scan_candidates(const PinHash& h, const float4* __restrict__ rec,
                                               float qx, float qy, float qz, TopK& tk) {
    const uint32_t B = (uint32_t)h.buffer_size;
    const uint32_t base = base_slot(qx, qy, qz, h.resolution, h.buffer_size);
    const float maxd2 = h.max_valid_dist2;
    const int Kc = h.num_cells;
    int nn = 0;
    for (int c0 = 0; c0 < Kc; c0 += CH) {
        int gi[CH];
#pragma unroll
        for (int t = 0; t < CH; ++t) {
            gi[t] = -1;
            if (c0 + t < Kc) {
                uint32_t s = base + (uint32_t)h.cells[4 * (c0 + t) + 3];
                s = s >= B ? s - B : s;
                gi[t] = h.table[s];
            }
        }
        float4 r[CH];
#pragma unroll
        for (int t = 0; t < CH; ++t) {
            r[t] = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
            if (gi[t] >= 0) r[t] = rec[gi[t]];
        }
#pragma unroll
        for (int t = 0; t < CH; ++t) {
            const int id = __float_as_int(r[t].w);
            if (gi[t] >= 0 && id != -1) {
                const float d2 = dist2(r[t].x, r[t].y, r[t].z, qx, qy, qz);
                if (d2 <= maxd2) {
                    ++nn;
                    tk.insert(d2, gi[t]);
                }
            }
        }
    }
    return nn;
}

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

// R(q) g: transpose of the passive rotation's Jacobian applied to g (d vec/dq = R(q)^T)
__device__ __forceinline__ void quat_rotate_active(float4 qt, float gx, float gy, float gz, float& ox, float& oy,
                                                   float& oz) {
    const float w = qt.x, x = qt.y, y = qt.z, z = qt.w;
    ox = (1.f - 2.f * (y * y + z * z)) * gx + 2.f * (x * y - w * z) * gy + 2.f * (x * z + w * y) * gz;
    oy = 2.f * (x * y + w * z) * gx + (1.f - 2.f * (x * x + z * z)) * gy + 2.f * (y * z - w * x) * gz;
    oz = 2.f * (x * z - w * y) * gx + 2.f * (y * z + w * x) * gy + (1.f - 2.f * (x * x + y * y)) * gz;
}

// Neighbour set of one query after the scan (weights and distance terms only; feature
// rows are streamed per neighbour by neighbour_input so they never stay live).
struct Neighbours {
    float w[kK];      // normalised IDW weights (0 for invalid)
    float u[kK];      // un-normalised 1/(d2+eps) (0 for invalid)
    float S;          // sum of u
    float pg[kK][3];  // q - global position (drives the distance gradient)
    int id[kK];       // feature row, -1 invalid
    int raw[kK];      // record id bits (flag = local position differs from the global one)
};

// neural_points.py:618-632 on the top-k: u = 1/(d2+eps), S = sum u, w = u/S (0 when invalid)
__device__ __forceinline__ void load_topk(const PinPoints& p, const TopK& tk, int nn, int nn_k, float qx, float qy,
                                          float qz, Neighbours& nb) {
    const float4* __restrict__ rec = (const float4*)p.records;
    float4 r[kK];
#pragma unroll
    for (int j = 0; j < kK; ++j) {
        r[j] = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
        if (j < nn_k && tk.g[j] >= 0) r[j] = rec[tk.g[j]];
    }
    float S = 0.f;
#pragma unroll
    for (int j = 0; j < kK; ++j) {
        const int raw = __float_as_int(r[j].w);
        const bool valid = j < nn_k && tk.g[j] >= 0;
        nb.raw[j] = raw;
        nb.id[j] = valid ? (raw & kIdMask) : -1;
        nb.u[j] = valid ? 1.0f / (tk.d[j] + kIdwEps) : 0.f;
        S = S + nb.u[j];
        nb.pg[j][0] = qx - r[j].x;
        nb.pg[j][1] = qy - r[j].y;
        nb.pg[j][2] = qz - r[j].z;
    }
    nb.S = S;
#pragma unroll
    for (int j = 0; j < kK; ++j) nb.w[j] = (nb.id[j] >= 0 && nn > 0) ? nb.u[j] / S : 0.f;
}

// Decoder input of neighbour j: feature row and neighbour vector q - p (local position,
// passively rotated by the point's quaternion after pgo: neural_points.py:577-608).
template <bool PGO>
__device__ __forceinline__ void neighbour_input(const PinPoints& p, const Neighbours& nb, int j, float qx, float qy,
                                                float qz, float (&x)[kD], float4& quat) {
    const int64_t id = nb.id[j];
    const float4* fr = (const float4*)(p.features + id * kF);
    const float4 f0 = fr[0], f1 = fr[1];
    x[0] = f0.x; x[1] = f0.y; x[2] = f0.z; x[3] = f0.w;
    x[4] = f1.x; x[5] = f1.y; x[6] = f1.z; x[7] = f1.w;
    if (nb.raw[j] & PIN_RECORD_UNFAITHFUL) {
        x[8] = qx - p.positions[3 * id];
        x[9] = qy - p.positions[3 * id + 1];
        x[10] = qz - p.positions[3 * id + 2];
    } else {
        x[8] = nb.pg[j][0];
        x[9] = nb.pg[j][1];
        x[10] = nb.pg[j][2];
    }
    quat = make_float4(1.f, 0.f, 0.f, 0.f);
    if (PGO) {
        quat = ((const float4*)p.orientations)[id];
        quat_rotate_passive(quat, x[8], x[9], x[10]);
    }
}

// Decoder forward fused with its input gradient (model/decoder.py:66-88):
//   sdf = s * (w2 . relu(W1 x + b1) + b2),  gx[i] = s * sum_c w2[c] 1[pre_c > 0] W1[c][OFF+i].
// One pass over the hidden units; weights are wave-uniform (scalar loads).
template <bool GRAD, int OFF, int NOUT>
__device__ __forceinline__ float mlp_sdf(const PinMlp& m, const float (&x)[kD], float (&gx)[NOUT]) {
    float out = 0.f;
#pragma unroll
    for (int i = 0; i < NOUT; ++i) gx[i] = 0.f;
#pragma unroll 8
    for (int c = 0; c < kH; ++c) {
        const float* wr = m.W1 + c * kD;
        float acc = 0.f;
#pragma unroll
        for (int i = 0; i < kD; ++i) acc = fmaf(wr[i], x[i], acc);
        const float pre = acc + m.b1[c];
        const float a = pre > 0.f ? m.W2[c] : 0.f;
        out = fmaf(a, pre, out);
        if (GRAD) {
#pragma unroll
            for (int i = 0; i < NOUT; ++i) gx[i] = fmaf(a, wr[OFF + i], gx[i]);
        }
    }
    if (GRAD) {
#pragma unroll
        for (int i = 0; i < NOUT; ++i) gx[i] *= m.sdf_scale;
    }
    return (out + m.b2[0]) * m.sdf_scale;
}

}  // namespace pin
