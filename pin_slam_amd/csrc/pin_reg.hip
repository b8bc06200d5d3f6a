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

// one block's partial accumulators -> partials[blockIdx.x * PIN_REG_NACC ..]
__device__ __forceinline__ void reg_block_partials(const float* __restrict__ pts, const float* __restrict__ sdf,
                                                   const float* __restrict__ grad, const int32_t* __restrict__ nn,
                                                   const float* __restrict__ std_, const float* __restrict__ label,
                                                   const float* __restrict__ weight, int64_t n, const PinRegParams& prm,
                                                   double* __restrict__ partials, uint8_t* __restrict__ valid_out) {
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
        float px, py, pz;
        int64_t src = i;   // the query's own index (labels, valid mask)
        if (prm.q4_points) {
            const float4 v = ((const float4*)pts)[i];
            px = v.x; py = v.y; pz = v.z;
            src = __float_as_int(v.w);
        } else {
            px = pts[3 * i]; py = pts[3 * i + 1]; pz = pts[3 * i + 2];
        }
        if (valid_out) valid_out[src] = valid ? 1 : 0;
        if (!valid) continue;
        const float sd = prm.div_grad_norm ? sdf[i] / gn : sdf[i];   // :335-336, "fix the overshot"
        const float r = sd - (label ? label[src] : 0.f);
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
    // block reduction, transposed through LDS: every thread's 31 accumulators land in column tid,
    // then 8 threads per accumulator sum 32 columns each (fixed order: part p takes columns
    // p, p + 8, ...) and a 3-step xor tree joins them.  (Per-accumulator shuffle trees were 372
    // ds_bpermute with ~190 waits per wave.)  Rows are padded to kRegBlock + 8 doubles: a wave's
    // 64 lanes (8 accumulators x 8 parts) then read dwords 16k + 2p (+16c) mod 64, every bank
    // pair twice -- the least a 64-lane 8-B read can do (unpadded, with contiguous column runs per
    // part, all 64 lanes hit one bank).
    __shared__ double red[PIN_REG_NACC][kRegBlock + 8];
    const int tid = threadIdx.x;
#pragma unroll
    for (int k = 0; k < PIN_REG_NACC; ++k) red[k][tid] = acc[k];
    __syncthreads();
    const int k = tid >> 3, part = tid & 7;
    double v = 0.0;
    if (k < PIN_REG_NACC) {
#pragma unroll 8
        for (int c = 0; c < kRegBlock / 8; ++c) v += red[k][part + 8 * c];
    }
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 4);
    if (k < PIN_REG_NACC && part == 0) partials[(int64_t)blockIdx.x * PIN_REG_NACC + k] = v;
}

__global__ void __launch_bounds__(kRegBlock)
k_reg_partials(const float* __restrict__ pts, const float* __restrict__ sdf, const float* __restrict__ grad,
               const int32_t* __restrict__ nn, const float* __restrict__ std_, const float* __restrict__ label,
               const float* __restrict__ weight, int64_t n, PinRegParams prm, double* __restrict__ partials,
               uint8_t* __restrict__ valid_out) {
    reg_block_partials(pts, sdf, grad, nn, std_, label, weight, n, prm, partials, valid_out);
}

// out[k] = sum of the block partials in a fixed order: thread t serves accumulator t / 8
// (31 x 8 = 248 threads), strided partial sums over the blocks, then a shuffle tree over
// the 8 lanes of each accumulator
// fixed-order sum of the block partials: thread (k, l) sums blocks l, l + 8, ... of accumulator k,
// then a shuffle tree over the 8 lanes
__device__ __forceinline__ double reg_final_sum(const double* __restrict__ partials, int nblk, int k, int l) {
    double v = 0.0;
    if (k < PIN_REG_NACC) {
#pragma unroll 8
        for (int b = l; b < nblk; b += 8) v += partials[(int64_t)b * PIN_REG_NACC + k];
    }
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 4);
    return v;
}

__global__ void __launch_bounds__(256) k_reg_final(const double* __restrict__ partials, int nblk,
                                                   double* __restrict__ out) {
    const int k = threadIdx.x >> 3, l = threadIdx.x & 7;
    const double v = reg_final_sum(partials, nblk, k, l);
    if (k < PIN_REG_NACC && l == 0) out[k] = v;
}

// transform_torch (utils/tools.py:386-399): [p, 1] @ T^T in f32 with T cast to f32, as the fma
// chain x, y, z then + t (the same arithmetic as pin_sample_rays' world copy)
__global__ void __launch_bounds__(kRegBlock)
k_transform_points(const float* __restrict__ src, int64_t n, const double* __restrict__ T, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * kRegBlock + threadIdx.x;
    if (i >= n) return;
    float t[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) t[e] = (float)T[e];
    const float px = src[3 * i], py = src[3 * i + 1], pz = src[3 * i + 2];
#pragma unroll
    for (int a = 0; a < 3; ++a) out[3 * i + a] = fmaf(pz, t[4 * a + 2], fmaf(py, t[4 * a + 1], px * t[4 * a])) + t[4 * a + 3];
}

// The same transform written into tile-sorted query rows in place: row k = {T src[i], bits(i)}
// with i = bits(q4[k].w) kept.  The tracking loop sorts its source cloud once (pin_query_sort) and
// re-poses the sorted rows every later iteration: the points move by the pose increment only, the
// order is a locality hint (results do not depend on it), and the two sort launches are saved.
__global__ void __launch_bounds__(kRegBlock)
k_transform_sorted(const float* __restrict__ src, int64_t n, const double* __restrict__ T, float4* __restrict__ q4) {
    const int64_t k = (int64_t)blockIdx.x * kRegBlock + threadIdx.x;
    if (k >= n) return;
    float t[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) t[e] = (float)T[e];
    const float w = q4[k].w;
    int i = __float_as_int(w);
    i = i < 0 || i >= n ? 0 : i;   // rows always come from pin_query_sort; never read outside src
    const float px = src[3 * (int64_t)i], py = src[3 * (int64_t)i + 1], pz = src[3 * (int64_t)i + 2];
    float o[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) o[a] = fmaf(pz, t[4 * a + 2], fmaf(py, t[4 * a + 1], px * t[4 * a])) + t[4 * a + 3];
    q4[k] = make_float4(o[0], o[1], o[2], w);
}

// implicit_reg's solve on the device (utils/tracker.py:483-496, expmap :580-589) and the tracking
// loop's bookkeeping of one iteration (:115, :132-133): from the accumulators of
// pin_reg_normal_eq, N = s sum w J^T J, g = -s sum w r J with s = n / (2 sum w) (the w /= 2 mean(w)
// of :394), N += lambda diag(N), t = N^-1 g (f64 Gaussian elimination, partial pivoting),
// dT = [expmap(t[0:3]) | t[3:6]], pose_out = dT pose_in.  One thread.
__device__ void reg_solve_body(const double* __restrict__ acc, double lm_lambda, const double* __restrict__ pose_in,
                               double* __restrict__ dT, double* __restrict__ pose_out, double* __restrict__ status) {
    const double s_w = acc[0], s_r = acc[1], cnt = acc[3];
    status[0] = cnt;
    status[1] = cnt > 0.0 ? s_r / cnt * 100.0 : 0.0;
    double D[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    double rot_deg = 0.0, tran = 0.0;
    const bool solve = cnt >= 10.0;   // :310-312 returns the identity below 10 valid points
    if (solve) {
        const double sc = cnt / (2.0 * s_w);
        double A[6][7];
        int k = 4;
        for (int a = 0; a < 6; ++a)
            for (int b = a; b < 6; ++b) {
                A[a][b] = A[b][a] = acc[k++] * sc;
            }
        for (int a = 0; a < 6; ++a) {
            A[a][a] += lm_lambda * A[a][a];
            A[a][6] = -acc[25 + a] * sc;
        }
        for (int c = 0; c < 6; ++c) {            // forward elimination with partial pivoting
            int piv = c;
            for (int r = c + 1; r < 6; ++r)
                if (fabs(A[r][c]) > fabs(A[piv][c])) piv = r;
            if (piv != c)
                for (int e = 0; e < 7; ++e) {
                    const double tmp = A[c][e];
                    A[c][e] = A[piv][e];
                    A[piv][e] = tmp;
                }
            for (int r = c + 1; r < 6; ++r) {
                const double f = A[r][c] / A[c][c];
                for (int e = c; e < 7; ++e) A[r][e] -= f * A[c][e];
            }
        }
        double t[6];
        for (int r = 5; r >= 0; --r) {
            double v = A[r][6];
            for (int e = r + 1; e < 6; ++e) v -= A[r][e] * t[e];
            t[r] = v / A[r][r];
        }
        // expmap: R = I + S sin(angle) + S^2 (1 - cos(angle)), S = skew(axis)
        const double angle = sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
        const double ax = t[0] / angle, ay = t[1] / angle, az = t[2] / angle;
        const double S[3][3] = {{0.0, -az, ay}, {az, 0.0, -ax}, {-ay, ax, 0.0}};
        const double sn = sin(angle), cs = 1.0 - cos(angle);
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) {
                double s2 = 0.0;
                for (int e = 0; e < 3; ++e) s2 += S[a][e] * S[e][b];
                D[4 * a + b] = (a == b ? 1.0 : 0.0) + S[a][b] * sn + s2 * cs;
            }
        D[3] = t[3];
        D[7] = t[4];
        D[11] = t[5];
        rot_deg = acos((D[0] + D[5] + D[10] - 1.0) / 2.0) * 180.0 / 3.141592653589793;   // :591-598
        tran = sqrt(t[3] * t[3] + t[4] * t[4] + t[5] * t[5]);
    }
    for (int e = 0; e < 16; ++e) dT[e] = D[e];
    if (pose_in && pose_out) {
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 4; ++b) {
                double v = 0.0;
                for (int e = 0; e < 4; ++e) v += D[4 * a + e] * pose_in[4 * e + b];
                pose_out[4 * a + b] = v;
            }
    }
    status[2] = rot_deg;
    status[3] = tran;
    status[4] = solve ? 1.0 : 0.0;
}

__global__ void k_reg_solve(const double* __restrict__ acc, double lm_lambda, const double* __restrict__ pose_in,
                            double* __restrict__ dT, double* __restrict__ pose_out, double* __restrict__ status) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    reg_solve_body(acc, lm_lambda, pose_in, dT, pose_out, status);
}

// The registration step's reductions and solve in ONE launch: every block writes its partials, the
// last block to finish (ticket on a counter that wraps back to zero) sums them in the fixed order of
// k_reg_final (bitwise the same accumulators) and runs the solve -- two launches fewer per
// iteration of the tracking loop.
__global__ void __launch_bounds__(kRegBlock)
k_reg_step(const float* __restrict__ pts, const float* __restrict__ sdf, const float* __restrict__ grad,
           const int32_t* __restrict__ nn, const float* __restrict__ std_, const float* __restrict__ label,
           int64_t n, PinRegParams prm, double* __restrict__ partials, unsigned* __restrict__ counter,
           double* __restrict__ acc, double lm_lambda, const double* __restrict__ pose_in, double* __restrict__ dT,
           double* __restrict__ pose_out, double* __restrict__ status) {
    reg_block_partials(pts, sdf, grad, nn, std_, label, nullptr, n, prm, partials, nullptr);
    __shared__ int last;
    __shared__ double s_acc[PIN_REG_NACC];
    // hand-off of the block partials (MI355X_MICROARCH.md, inter-workgroup visibility, valid form):
    // storing waves wait for their stores, one lane releases at agent scope (the L2 write-back),
    // waits for it, then takes the ticket; the last block's lane 0 acquires (its CU's L1
    // invalidated) before the block's plain loads.  One fence per block, not per thread.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = atomicInc(counter, gridDim.x - 1) == gridDim.x - 1;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    if (!last) return;
    const int k = threadIdx.x >> 3, l = threadIdx.x & 7;
    const double v = reg_final_sum(partials, gridDim.x, k, l);
    if (k < PIN_REG_NACC && l == 0) {
        acc[k] = v;
        s_acc[k] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) reg_solve_body(s_acc, lm_lambda, pose_in, dT, pose_out, status);
}

}  // namespace

extern "C" {

int pin_transform_points(const float* points, int64_t n, const double* pose, float* out, void* stream) {
    if (n < 0 || (n > 0 && (!points || !pose || !out))) return PIN_ERR_ARG;
    if (n == 0) return PIN_OK;
    hipLaunchKernelGGL(k_transform_points, dim3((unsigned)((n + kRegBlock - 1) / kRegBlock)), dim3(kRegBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), points, n, pose, out);
    return hipGetLastError() == hipSuccess ? PIN_OK : PIN_ERR_HIP;
}

int pin_transform_points_sorted(const float* points, int64_t n, const double* pose, float* q4, void* stream) {
    if (n < 0 || n > INT32_MAX || (n > 0 && (!points || !pose || !q4))) return PIN_ERR_ARG;
    if (n == 0) return PIN_OK;
    hipLaunchKernelGGL(k_transform_sorted, dim3((unsigned)((n + kRegBlock - 1) / kRegBlock)), dim3(kRegBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), points, n, pose, (float4*)q4);
    return hipGetLastError() == hipSuccess ? PIN_OK : PIN_ERR_HIP;
}

int pin_reg_solve(const double* acc, double lm_lambda, const double* pose_in, double* delta_pose, double* pose_out,
                  double* status, void* stream) {
    if (!acc || !delta_pose || !status || (pose_out && !pose_in)) return PIN_ERR_ARG;
    hipLaunchKernelGGL(k_reg_solve, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), acc, lm_lambda,
                       pose_in, delta_pose, pose_out, status);
    return hipGetLastError() == hipSuccess ? PIN_OK : PIN_ERR_HIP;
}

int pin_reg_step(const float* points, const float* sdf, const float* grad, const int32_t* nn_count,
                 const float* sdf_std, const float* sdf_label, int64_t n, const PinRegParams* prm, double* workspace,
                 double* acc, double lm_lambda, const double* pose_in, double* delta_pose, double* pose_out,
                 double* status, void* stream) {
    if (!prm || !acc || !workspace || !delta_pose || !status || (pose_out && !pose_in) || n < 0) return PIN_ERR_ARG;
    if (n > 0 && (!points || !sdf || !grad || !nn_count)) return PIN_ERR_ARG;
    const int nblk = (int)std::min<int64_t>(std::max<int64_t>((n + kRegBlock - 1) / kRegBlock, 1), kRegMaxBlocks);
    unsigned* counter = (unsigned*)(workspace + kRegMaxBlocks * PIN_REG_NACC);
    hipLaunchKernelGGL(k_reg_step, dim3(nblk), dim3(kRegBlock), 0, reinterpret_cast<hipStream_t>(stream), points, sdf,
                       grad, nn_count, sdf_std, sdf_label, n, *prm, workspace, counter, acc, lm_lambda, pose_in,
                       delta_pose, pose_out, status);
    return hipGetLastError() == hipSuccess ? PIN_OK : PIN_ERR_HIP;
}

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
