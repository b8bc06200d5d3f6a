// pin_sample.hip -- training-sample generation along the scan rays (utils/data_sampler.py:20-192)
// fused with the pose transform of utils/mapper.py:133-215 (transform_torch, utils/tools.py:386-399).
//
// One thread per output row.  Row r = i * A + j is sample j of ray i in the reference's final
// ray-wise order (data_sampler.py:165-171): j = 0 the measured point, then surface_n surface
// samples, free_front_n free-space samples in front, free_behind_n behind.  Every elementwise
// expression follows the reference's op order in f32 (scalar-only subexpressions were evaluated
// by Python in double and are passed pre-rounded), so given the same random draws the outputs
// are the reference's.  The draws are the caller's torch.randn / torch.rand tensors, drawn in
// the reference's order (surface randn [S*N], front rand [F*N], behind rand [B*N]; part-major,
// draw k*N + i belongs to ray i).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pin_slam_amd.h"

namespace {

constexpr int kSampleBlock = 256;

__global__ void __launch_bounds__(kSampleBlock)
k_sample_rays(const float* __restrict__ pts, int64_t n, const float* __restrict__ rn_surface,
              const float* __restrict__ r_front, const float* __restrict__ r_behind, PinSampleCfg c,
              float* __restrict__ coord, float* __restrict__ sdf_label, float* __restrict__ weight,
              float* __restrict__ global_coord) {
    const int A = 1 + c.surface_n + c.front_n + c.behind_n;
    const int64_t r = (int64_t)blockIdx.x * kSampleBlock + threadIdx.x;
    if (r >= n * A) return;
    const int64_t i = r / A;
    const int j = (int)(r - i * A);
    const float x = pts[3 * i], y = pts[3 * i + 1], z = pts[3 * i + 2];
    const float d = sqrtf(fmaf(z, z, fmaf(y, y, x * x)));   // torch.linalg.norm(dim=1) on the CPU
    float ratio, disp;
    bool surface = true;
    if (j == 0) {                                       // :45-46
        ratio = 1.0f;
        disp = 0.0f;
    } else if (j <= c.surface_n) {                      // :50-53
        disp = rn_surface[(int64_t)(j - 1) * n + i] * c.surface_range;
        ratio = disp / d + 1.0f;
    } else if (j <= c.surface_n + c.front_n) {          // :72-78
        // python_scalar / tensor is Tensor.__rtruediv__ = reciprocal(tensor) * scalar
        const float fmax = 1.0f - (1.0f / d) * c.two_range;
        const float fdiff = fmax - c.front_min_ratio;
        ratio = r_front[(int64_t)(j - 1 - c.surface_n) * n + i] * fdiff + c.front_min_ratio;
        disp = (ratio - 1.0f) * d;
        surface = false;
    } else {                                            // :85-91
        const float bmax = (1.0f / d) * c.end_dist + 1.0f;
        const float bmin = 1.0f + (1.0f / d) * c.two_range;
        const float bdiff = bmax - bmin;
        ratio = r_behind[(int64_t)(j - 1 - c.surface_n - c.front_n) * n + i] * bdiff + bmin;
        disp = (ratio - 1.0f) * d;
        surface = false;
    }
    const float px = x * ratio, py = y * ratio, pz = z * ratio;   // :106
    float w = 1.0f;                                               // :117
    if (c.dist_weight_on && surface)                              // :120-121
        w = c.dist_weight_base - (d / c.max_range) * c.dist_weight_scale;
    if (c.behind_dropoff_on) {                                    // :125-134
        float dw = (c.dropoff_max - disp) / c.dropoff_diff;
        dw = fminf(fmaxf(dw, 0.0f), 1.0f);
        dw = dw * 0.8f + 0.2f;
        w = w * dw;
    }
    if (!surface) w = w * -1.0f;                                  // :137
    coord[3 * r] = px;
    coord[3 * r + 1] = py;
    coord[3 * r + 2] = pz;
    sdf_label[r] = disp * -1.0f;                                  // :144, :167
    weight[r] = w;
    if (global_coord) {   // transform_torch: [p, 1] @ T^T in f32 (T cast to f32), the CPU sgemm's fma chain
        const float* T = c.pose;
#pragma unroll
        for (int a = 0; a < 3; ++a)
            global_coord[3 * r + a] = fmaf(pz, T[4 * a + 2], fmaf(py, T[4 * a + 1], px * T[4 * a])) + T[4 * a + 3];
    }
}

}  // namespace

extern "C" {

int pin_sample_rays(const float* points, int64_t n, const float* randn_surface, const float* rand_front,
                    const float* rand_behind, const PinSampleCfg* cfg, float* coord, float* sdf_label, float* weight,
                    float* global_coord, void* stream) {
    if (!cfg || n < 0 || cfg->surface_n < 0 || cfg->front_n < 0 || cfg->behind_n < 0) return PIN_ERR_ARG;
    if (n == 0) return PIN_OK;
    if (!points || !coord || !sdf_label || !weight) return PIN_ERR_ARG;
    if ((cfg->surface_n && !randn_surface) || (cfg->front_n && !rand_front) || (cfg->behind_n && !rand_behind))
        return PIN_ERR_ARG;
    if (global_coord && !cfg->pose) return PIN_ERR_ARG;
    const int64_t rows = n * (1 + cfg->surface_n + cfg->front_n + cfg->behind_n);
    hipLaunchKernelGGL(k_sample_rays, dim3((unsigned)((rows + kSampleBlock - 1) / kSampleBlock)), dim3(kSampleBlock),
                       0, reinterpret_cast<hipStream_t>(stream), points, n, randn_surface, rand_front, rand_behind,
                       *cfg, coord, sdf_label, weight, global_coord);
    return hipGetLastError() == hipSuccess ? PIN_OK : PIN_ERR_HIP;
}

}  // extern "C"

// ------------------------------------------------------------------ deskewing (utils/tools.py:540-567)
// Per point: s = (ts - min) / (max - min) - ts_mid; R(s) = exp(s log R_pose) (roma.rotmat_slerp from
// the identity: the relative rotation's rotation vector scaled by s, Rodrigues), t(s) = s t_pose;
// p <- R(s) p + t(s) for the first three channels of each row, in place (the reference aliases
// its input).  log R is taken through the unit quaternion (largest-component branch), as roma
// does, then 2 atan2(|v|, w) v / |v|.
namespace {

__device__ __forceinline__ void rotmat_to_rotvec(const float* T, float& wx, float& wy, float& wz) {
    const float r00 = T[0], r01 = T[1], r02 = T[2], r10 = T[4], r11 = T[5], r12 = T[6], r20 = T[8], r21 = T[9],
                r22 = T[10];
    const float tr = r00 + r11 + r22;
    float qw, qx, qy, qz;
    if (tr >= r00 && tr >= r11 && tr >= r22) {
        qw = 1.0f + tr; qx = r21 - r12; qy = r02 - r20; qz = r10 - r01;
    } else if (r00 >= r11 && r00 >= r22) {
        qw = r21 - r12; qx = 1.0f + r00 - r11 - r22; qy = r01 + r10; qz = r02 + r20;
    } else if (r11 >= r22) {
        qw = r02 - r20; qx = r01 + r10; qy = 1.0f + r11 - r00 - r22; qz = r12 + r21;
    } else {
        qw = r10 - r01; qx = r02 + r20; qy = r12 + r21; qz = 1.0f + r22 - r00 - r11;
    }
    const float qn = sqrtf(qw * qw + qx * qx + qy * qy + qz * qz);
    qw /= qn; qx /= qn; qy /= qn; qz /= qn;
    if (qw < 0.f) { qw = -qw; qx = -qx; qy = -qy; qz = -qz; }
    const float vn = sqrtf(qx * qx + qy * qy + qz * qz);
    const float ang = 2.0f * atan2f(vn, qw);
    const float k = vn > 1e-12f ? ang / vn : 2.0f;   // small angle: 2 / w with w ~ 1
    wx = qx * k; wy = qy * k; wz = qz * k;
}

__global__ void __launch_bounds__(kSampleBlock)
k_deskew(float* __restrict__ pts, int64_t n, int64_t stride, const float* __restrict__ ts,
         const float* __restrict__ minmax, const float* __restrict__ pose, float ts_mid) {
    const int64_t i = (int64_t)blockIdx.x * kSampleBlock + threadIdx.x;
    if (i >= n) return;
    float wx, wy, wz;
    rotmat_to_rotvec(pose, wx, wy, wz);
    const float s = (ts[i] - minmax[0]) / (minmax[1] - minmax[0]) - ts_mid;
    const float ax = s * wx, ay = s * wy, az = s * wz;
    const float th2 = ax * ax + ay * ay + az * az;
    const float th = sqrtf(th2);
    float a, b;   // R = I + a [w]x + b [w]x^2
    if (th < 1e-4f) {
        a = 1.0f - th2 / 6.0f;
        b = 0.5f - th2 / 24.0f;
    } else {
        a = sinf(th) / th;
        b = (1.0f - cosf(th)) / th2;
    }
    float* p = pts + i * stride;
    const float x = p[0], y = p[1], z = p[2];
    // [w]x p = w x p ; [w]x^2 p = w x (w x p)
    const float cx = ay * z - az * y, cy = az * x - ax * z, cz = ax * y - ay * x;
    const float dx = ay * cz - az * cy, dy = az * cx - ax * cz, dz = ax * cy - ay * cx;
    p[0] = x + a * cx + b * dx + s * pose[3];
    p[1] = y + a * cy + b * dy + s * pose[7];
    p[2] = z + a * cz + b * dz + s * pose[11];
}

}  // namespace

extern "C" int pin_deskew(float* points, int64_t n, int64_t stride, const float* ts, const float* ts_minmax,
                          const float* pose, float ts_mid_pose, void* stream) {
    if (n < 0 || stride < 3) return PIN_ERR_ARG;
    if (n == 0) return PIN_OK;
    if (!points || !ts || !ts_minmax || !pose) return PIN_ERR_ARG;
    hipLaunchKernelGGL(k_deskew, dim3((unsigned)((n + kSampleBlock - 1) / kSampleBlock)), dim3(kSampleBlock), 0,
                       reinterpret_cast<hipStream_t>(stream), points, n, stride, ts, ts_minmax, pose, ts_mid_pose);
    return hipGetLastError() == hipSuccess ? PIN_OK : PIN_ERR_HIP;
}
