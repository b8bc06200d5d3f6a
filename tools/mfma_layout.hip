// Checks the operand/accumulator layout assumed by mlp_sdf_mfma16 (pin_device.h) for
// v_mfma_f32_16x16x32_f16 and v_mfma_f32_16x16x16_f16: lane l supplies A row l%16 and B column
// l%16 with K-slots 8(l/16)..+7 (x16: 4(l/16)..+3); D row 4(l/16)+r, column l%16.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k(const float* A, const float* B, const float* A2, const float* B2, float* D, float* D2) {
    const int l = threadIdx.x, i = l & 15, g = l >> 4;
    f16x8 a, b;
    for (int s = 0; s < 8; ++s) { a[s] = (_Float16)A[i * 32 + 8 * g + s]; b[s] = (_Float16)B[(8 * g + s) * 16 + i]; }
    f32x4 d = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, (f32x4){0, 0, 0, 0}, 0, 0, 0);
    f16x4 a4, b4;
    for (int s = 0; s < 4; ++s) { a4[s] = (_Float16)A2[i * 16 + 4 * g + s]; b4[s] = (_Float16)B2[(4 * g + s) * 16 + i]; }
    f32x4 d2 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, (f32x4){0, 0, 0, 0}, 0, 0, 0);
    for (int r = 0; r < 4; ++r) { D[(4 * g + r) * 16 + i] = d[r]; D2[(4 * g + r) * 16 + i] = d2[r]; }
}

int main() {
    float hA[16 * 32], hB[32 * 16], hA2[256], hB2[256], hD[256], hD2[256];
    for (int e = 0; e < 512; ++e) { hA[e] = (float)((e * 7) % 13 - 6); hB[e] = (float)((e * 5) % 11 - 5); }
    for (int e = 0; e < 256; ++e) { hA2[e] = (float)((e * 3) % 7 - 3); hB2[e] = (float)((e * 11) % 9 - 4); }
    float *A, *B, *A2, *B2, *D, *D2;
    hipMalloc(&A, 2048); hipMalloc(&B, 2048); hipMalloc(&A2, 1024); hipMalloc(&B2, 1024);
    hipMalloc(&D, 1024); hipMalloc(&D2, 1024);
    hipMemcpy(A, hA, 2048, hipMemcpyHostToDevice); hipMemcpy(B, hB, 2048, hipMemcpyHostToDevice);
    hipMemcpy(A2, hA2, 1024, hipMemcpyHostToDevice); hipMemcpy(B2, hB2, 1024, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, A, B, A2, B2, D, D2);
    hipMemcpy(hD, D, 1024, hipMemcpyDeviceToHost); hipMemcpy(hD2, D2, 1024, hipMemcpyDeviceToHost);
    int bad = 0, bad2 = 0;
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) {
            float s = 0, s2 = 0;
            for (int kk = 0; kk < 32; ++kk) s += hA[i * 32 + kk] * hB[kk * 16 + j];
            for (int kk = 0; kk < 16; ++kk) s2 += hA2[i * 16 + kk] * hB2[kk * 16 + j];
            if (hD[i * 16 + j] != s) { if (bad < 5) printf("x32 D[%d][%d] %g want %g\n", i, j, hD[i * 16 + j], s); ++bad; }
            if (hD2[i * 16 + j] != s2) { if (bad2 < 5) printf("x16 D[%d][%d] %g want %g\n", i, j, hD2[i * 16 + j], s2); ++bad2; }
        }
    printf("16x16x32 f16 mismatches %d, 16x16x16 f16 mismatches %d\n", bad, bad2);
    return bad || bad2;
}
