// pin_reg.hip -- point-to-implicit registration normal equations (utils/tracker.py:277-520).
//
// After the fused query has produced sdf / dsdf/dq / nn_count (/ std) for every source
// point, one pass over the points forms, for the valid ones (:305),
//   r_i = sdf_i - label_i,  w_i = w_res(r_i) * w_grad(|g_i| - 1)      (Geman-McClure, :353-354)
//   J_i = [p_i x g_i, g_i]                                            (:470-471)
// and accumulates in f64
//   S_w = sum w_i, S_r = sum |r_i|, S_wr2 = sum w_i r_i^2, n_valid,
//   N'  = sum w_i J_i^T J_i (21 unique entries),  g' = sum w_i r_i J_i.
// The reference's normalisation w /= 2 mean(w) (:394) is the scalar count / (2 S_w) applied
// on the host.  Partials are per block and summed in a fixed order by a second one-block
// kernel, so the result is bitwise reproducible run to run.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "pin_device.h"

namespace {

constexpr int kRegBlock = 256;
constexpr int kRegMaxBlocks = 256;

__device__ __forceinline__ double wave_sum(double v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
    return v;
}

__global__ void __launch_bounds__(kRegBlock)
k_reg_partials(const float* __restrict__ pts, const float* __restrict__ sdf, const float* __restrict__ grad,
               const int32_t* __restrict__ nn, const float* __restrict__ std_, const float* __restrict__ label,
               const float* __restrict__ weight, int64_t n, PinRegParams prm, double* __restrict__ partials,
               uint8_t* __restrict__ valid_out) {
    double acc[PIN_REG_NACC];
#pragma unroll
    for (int k = 0; k < PIN_REG_NACC; ++k) acc[k] = 0.0;
    const int64_t stride = (int64_t)gridDim.x * kRegBlock;
    for (int64_t i = (int64_t)blockIdx.x * kRegBlock + threadIdx.x; i < n; i += stride) {
        const float gx = grad[3 * i], gy = grad[3 * i + 1], gz = grad[3 * i + 2];
        const float gn = sqrtf((gx * gx + gy * gy) + gz * gz);
        bool valid = true;
        if (!weight) {
            valid = nn[i] >= prm.min_nn_count && gn < prm.max_grad_norm && gn > prm.min_grad_norm;
            if (std_) valid = valid && std_[i] < prm.max_sdf_std;
        }
        if (valid_out) valid_out[i] = valid ? 1 : 0;
        if (!valid) continue;
        const float sd = prm.div_grad_norm ? sdf[i] / gn : sdf[i];   // :335-336, "fix the overshot"
        const float r = sd - (label ? label[i] : 0.f);
        float w = 1.f;
        if (weight) {
            w = weight[i];
        } else if (prm.gm_grad > 0.f) {
            const float ga = gn - 1.f;
            const float t = prm.gm_grad / (prm.gm_grad * prm.gm_grad + ga * ga);
            w = w * (t * t);
        }
        if (!weight && prm.gm_dist > 0.f) {
            const float t = prm.gm_dist / (prm.gm_dist * prm.gm_dist + r * r);
            w = (t * t) * w;
        }
        const float px = pts[3 * i], py = pts[3 * i + 1], pz = pts[3 * i + 2];
        const double J[6] = {(double)(py * gz - pz * gy), (double)(pz * gx - px * gz), (double)(px * gy - py * gx),
                             (double)gx, (double)gy, (double)gz};
        const double wd = w, rd = r;
        acc[0] += wd;
        acc[1] += fabs(rd);
        acc[2] += wd * rd * rd;
        acc[3] += 1.0;
        int k = 4;
#pragma unroll
        for (int a = 0; a < 6; ++a)
#pragma unroll
            for (int b = a; b < 6; ++b) acc[k++] += wd * J[a] * J[b];
#pragma unroll
        for (int a = 0; a < 6; ++a) acc[25 + a] += wd * rd * J[a];
    }
    __shared__ double red[kRegBlock / 64][PIN_REG_NACC];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < PIN_REG_NACC; ++k) {
        const double v = wave_sum(acc[k]);
        if (lane == 0) red[wave][k] = v;
    }
    __syncthreads();
    if (threadIdx.x < PIN_REG_NACC) {
        double v = 0.0;
        for (int w = 0; w < kRegBlock / 64; ++w) v += red[w][threadIdx.x];
        partials[(int64_t)blockIdx.x * PIN_REG_NACC + threadIdx.x] = v;
    }
}

// out[k] = sum of the block partials in a fixed order: thread t serves accumulator t / 8
// (31 x 8 = 248 threads), strided partial sums over the blocks, then a shuffle tree over
// the 8 lanes of each accumulator
__global__ void __launch_bounds__(256) k_reg_final(const double* __restrict__ partials, int nblk,
                                                   double* __restrict__ out) {
    const int k = threadIdx.x >> 3, l = threadIdx.x & 7;
    double v = 0.0;
    if (k < PIN_REG_NACC)
        for (int b = l; b < nblk; b += 8) v += partials[(int64_t)b * PIN_REG_NACC + k];
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 4);
    if (k < PIN_REG_NACC && l == 0) out[k] = v;
}

}  // namespace

extern "C" {

int pin_reg_normal_eq(const float* points, const float* sdf, const float* grad, const int32_t* nn_count,
                      const float* sdf_std, const float* sdf_label, const float* weight, int64_t n,
                      const PinRegParams* prm, double* workspace, double* out, uint8_t* valid_out, void* stream) {
    if (!prm || !out || !workspace || n < 0) return PIN_ERR_ARG;
    if (n > 0 && (!points || !sdf || !grad || (!nn_count && !weight))) return PIN_ERR_ARG;
    const int nblk = (int)std::min<int64_t>(std::max<int64_t>((n + kRegBlock - 1) / kRegBlock, 1), kRegMaxBlocks);
    auto s = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_reg_partials, dim3(nblk), dim3(kRegBlock), 0, s, points, sdf, grad, nn_count, sdf_std,
                       sdf_label, weight, n, *prm, workspace, valid_out);
    hipLaunchKernelGGL(k_reg_final, dim3(1), dim3(256), 0, s, workspace, nblk, out);
    return hipGetLastError() == hipSuccess ? PIN_OK : PIN_ERR_HIP;
}

}  // extern "C"
