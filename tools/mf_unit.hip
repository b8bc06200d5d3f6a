// Unit check of mlp_sdf_mfma16 against the f32 VALU decoder on random decoders and inputs,
// one block of 4 waves (standalone: hipcc -I include -I pin_slam_amd/csrc tools/mf_unit.hip).
#include "../pin_slam_amd/csrc/pin_query.hip"
#include <cstdio>
#include <cstdlib>
#include <cmath>

__global__ void k_unit(const PinMlp m, const float* __restrict__ X, float* __restrict__ out) {
    __shared__ float s_mlp[kWSize];
    __shared__ uint4 s_pk[kPkBytes / 16];
    __shared__ float s_x16[kBlock / 64][kXsWave];
    for (int e = threadIdx.x; e < kPkBytes / 16; e += kBlock) s_pk[e] = ((const uint4*)m.packed)[e];
    MlpW mv = stage_mlp(m, s_mlp);   // ends with a barrier
    MlpW mm{nullptr, m.sdf_scale, s_x16[threadIdx.x >> 6], (const unsigned char*)s_pk};
    const int t = blockIdx.x * kBlock + threadIdx.x;
    float x[kD];
    for (int i = 0; i < kD; ++i) x[i] = X[t * kD + i];
    float g0[kD], g1[kD];
    const float s0 = mlp_sdf<true, 0, kD>(mv, x, g0);
    const float s1 = mlp_sdf_mfma16<true, 0, kD>(mm, x, g1);
    out[t * 24 + 0] = s0;
    out[t * 24 + 1] = s1;
    for (int i = 0; i < kD; ++i) { out[t * 24 + 2 + i] = g0[i]; out[t * 24 + 13 + i] = g1[i]; }
}

int main() {
    const int nb = 8, n = nb * kBlock;
    srand(1);
    auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
    float hW1[64 * 11], hb1[64], hW2[64], hb2[1];
    for (auto& v : hW1) v = 0.3f * rnd();
    for (auto& v : hb1) v = 0.3f * rnd();
    for (auto& v : hW2) v = 0.12f * rnd();
    hb2[0] = 0.05f;
    float* hX = (float*)malloc(n * kD * 4);
    for (int e = 0; e < n * kD; ++e) hX[e] = (e % kD < 8 ? 0.05f : 0.5f) * rnd();
    float *W1, *b1, *W2, *b2, *X, *out;
    void* pk;
    (void)hipMalloc(&W1, sizeof hW1); (void)hipMalloc(&b1, 256); (void)hipMalloc(&W2, 256); (void)hipMalloc(&b2, 4);
    (void)hipMalloc(&X, n * kD * 4); (void)hipMalloc(&out, n * 24 * 4); (void)hipMalloc(&pk, kPkBytes);
    (void)hipMemcpy(W1, hW1, sizeof hW1, hipMemcpyHostToDevice); (void)hipMemcpy(b1, hb1, 256, hipMemcpyHostToDevice);
    (void)hipMemcpy(W2, hW2, 256, hipMemcpyHostToDevice); (void)hipMemcpy(b2, hb2, 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(X, hX, n * kD * 4, hipMemcpyHostToDevice);
    PinMlp m{W1, b1, W2, b2, 1.0f, 0, pk};
    if (pin_mlp_pack(&m, pk, nullptr) != PIN_OK) { printf("pack failed\n"); return 1; }
    hipLaunchKernelGGL(k_unit, dim3(nb), dim3(kBlock), 0, 0, m, X, out);
    float* h = (float*)malloc(n * 24 * 4);
    (void)hipMemcpy(h, out, n * 24 * 4, hipMemcpyDeviceToHost);
    double es = 0, eg = 0;
    int bad = 0;
    for (int t = 0; t < n; ++t) {
        const double d = fabs(h[t * 24] - h[t * 24 + 1]);
        es = fmax(es, d);
        for (int i = 0; i < kD; ++i) eg = fmax(eg, fabs(h[t * 24 + 2 + i] - h[t * 24 + 13 + i]));
        if (d > 1e-5 && bad++ < 8) printf("t %d (lane %d) valu %g mfma %g\n", t, t & 63, h[t * 24], h[t * 24 + 1]);
    }
    printf("max |sdf diff| %g  max |grad diff| %g  bad %d / %d\n", es, eg, bad, n);
    return bad != 0;
}
