// pin_grid.hip -- the succinct occupancy grid that replaces the hash probes on the hot path.
//
// The reference finds candidates by hashing each neighbour cell into a 5e7-slot table
// (model/neural_points.py:465-476): 33 random probes into a 200-400 MB array per query,
// two thirds of them empty.  For a map whose table entries all sit at their point's own
// voxel slot (true after update / recreate_hash), the function cell -> table[slot(cell)]
// restricted to the candidates that can pass the distance test is the same as
// cell -> "the point whose own voxel is this cell and whose slot holds it", provided no
// two cells within the reachable window collide under the hash (checked on the host).
// That function is stored as
//   bricks[b]  = {bits lo, bits hi, prefix, 0}   4x4x4 cells per brick, one bit per cell
//   crec[r]    = 64-byte record of the r-th occupied cell in brick order
//                {x, y, z, bits(id)} {f0..f3} {f4..f7} {certainty, 0, 0, 0}
//   cgid[r]    = global point index of that record
// The bricks of a 1M-point surface map are ~2 MB: L2-resident on every XCD, so the
// probe phase costs L1/L2 hits and only real candidates touch HBM (one line each).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "pin_device.h"

using namespace pin;

namespace {

constexpr int kScanItems = 16;  // bricks per thread in the prefix scan

inline dim3 grid_for(int64_t n, int per = kBlock) { return dim3((unsigned)((n + per - 1) / per)); }
inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }
inline int launch_status() { return hipGetLastError() == hipSuccess ? PIN_OK : PIN_ERR_HIP; }

__device__ __forceinline__ bool own_cell(const float* __restrict__ pos, int64_t g, float res, int64_t B,
                                         const int32_t* __restrict__ table, const PinGridDims& d, int64_t& brick,
                                         int& bit) {
    const float x = pos[3 * g], y = pos[3 * g + 1], z = pos[3 * g + 2];
    if (table[base_slot(x, y, z, res, B)] != (int)g) return false;
    const int64_t lx = (int64_t)floorf(x / res) - d.ox;
    const int64_t ly = (int64_t)floorf(y / res) - d.oy;
    const int64_t lz = (int64_t)floorf(z / res) - d.oz;
    if (lx < 0 || ly < 0 || lz < 0 || lx >= 4ll * d.nbx || ly >= 4ll * d.nby || lz >= 4ll * d.nbz) return false;
    brick = ((lz >> 2) * d.nby + (ly >> 2)) * (int64_t)d.nbx + (lx >> 2);
    bit = (int)(((lx & 3) << 4) | ((ly & 3) << 2) | (lz & 3));
    return true;
}

__global__ void __launch_bounds__(kBlock)
k_grid_mark(const float* __restrict__ pos, int64_t M, float res, const int32_t* __restrict__ table, int64_t B,
            PinGridDims d, uint32_t* __restrict__ bricks, unsigned long long* __restrict__ marked) {
    const int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    int64_t brick;
    int bit;
    const bool own = g < M && own_cell(pos, g, res, B, table, d, brick, bit);
    if (own) atomicOr(bricks + 4 * brick + (bit >> 5), 1u << (bit & 31));
    const unsigned long long ball = __ballot(own);
    if ((threadIdx.x & 63) == 0 && ball) atomicAdd(marked, (unsigned long long)__popcll(ball));
}

__global__ void __launch_bounds__(kBlock)
k_table_count(const int32_t* __restrict__ table, int64_t B, unsigned long long* __restrict__ count) {
    int64_t c = 0;
    const int64_t stride = (int64_t)gridDim.x * kBlock * 4;
    for (int64_t i = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 4; i < B; i += stride) {
        if (i + 3 < B) {
            const int4 v = *(const int4*)(table + i);
            c += (v.x >= 0) + (v.y >= 0) + (v.z >= 0) + (v.w >= 0);
        } else {
            for (int64_t k = i; k < B; ++k) c += table[k] >= 0;
        }
    }
    for (int off = 32; off > 0; off >>= 1) c += __shfl_down(c, off);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(count, (unsigned long long)c);
}

// exclusive prefix of per-brick popcounts: block partial sums, one-block scan of the
// partials, then the per-brick pass
__global__ void __launch_bounds__(kBlock)
k_scan_partials(const uint32_t* __restrict__ bricks, int64_t nb, uint32_t* __restrict__ part) {
    __shared__ uint32_t red[kBlock / 64];
    const int64_t b0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * kScanItems;
    uint32_t s = 0;
    for (int k = 0; k < kScanItems; ++k) {
        const int64_t b = b0 + k;
        if (b < nb) s += __popc(bricks[4 * b]) + __popc(bricks[4 * b + 1]);
    }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += red[w];
        part[blockIdx.x] = t;
    }
}

__global__ void __launch_bounds__(1024) k_scan_block_sums(uint32_t* __restrict__ part, int64_t np) {
    __shared__ uint32_t buf[1024];
    uint32_t carry = 0;
    for (int64_t base = 0; base < np; base += 1024) {
        const int64_t i = base + threadIdx.x;
        const uint32_t v = i < np ? part[i] : 0;
        buf[threadIdx.x] = v;
        __syncthreads();
        for (int off = 1; off < 1024; off <<= 1) {
            const uint32_t t = threadIdx.x >= off ? buf[threadIdx.x - off] : 0;
            __syncthreads();
            buf[threadIdx.x] += t;
            __syncthreads();
        }
        if (i < np) part[i] = carry + buf[threadIdx.x] - v;  // exclusive
        const uint32_t tot = buf[1023];
        __syncthreads();
        carry += tot;
    }
}

__global__ void __launch_bounds__(kBlock)
k_scan_apply(uint32_t* __restrict__ bricks, int64_t nb, const uint32_t* __restrict__ part) {
    __shared__ uint32_t wsum[kBlock / 64];
    const int64_t b0 = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * kScanItems;
    uint32_t cnt[kScanItems];
    uint32_t s = 0;
    for (int k = 0; k < kScanItems; ++k) {
        const int64_t b = b0 + k;
        cnt[k] = b < nb ? __popc(bricks[4 * b]) + __popc(bricks[4 * b + 1]) : 0;
        s += cnt[k];
    }
    // exclusive scan of s across the block
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t inc = s;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(inc, off);
        if (lane >= off) inc += t;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    uint32_t wbase = 0;
    for (int w = 0; w < wave; ++w) wbase += wsum[w];
    uint32_t run = part[blockIdx.x] + wbase + inc - s;
    for (int k = 0; k < kScanItems; ++k) {
        const int64_t b = b0 + k;
        if (b < nb) bricks[4 * b + 2] = run;
        run += cnt[k];
    }
}

__global__ void __launch_bounds__(kBlock)
k_grid_fill(const float* __restrict__ pos, int64_t M, float res, const int32_t* __restrict__ table, int64_t B,
            PinGridDims d, const uint32_t* __restrict__ bricks, const float4* __restrict__ rec,
            const float* __restrict__ feat, const float* __restrict__ cert, float4* __restrict__ crec,
            int32_t* __restrict__ cgid) {
    const int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (g >= M) return;
    int64_t brick;
    int bit;
    if (!own_cell(pos, g, res, B, table, d, brick, bit)) return;
    const uint4 w = *(const uint4*)(bricks + 4 * brick);
    const uint64_t bits = ((uint64_t)w.y << 32) | w.x;
    const uint32_t r = w.z + (uint32_t)__popcll(bits & ((1ull << bit) - 1ull));
    const float4 rc = rec[g];
    const int id = __float_as_int(rc.w);
    float4 f0 = make_float4(0.f, 0.f, 0.f, 0.f), f1 = f0, c = f0;
    if (id != -1 && feat) {
        const int64_t row = id & kIdMask;
        f0 = ((const float4*)feat)[2 * row];
        f1 = ((const float4*)feat)[2 * row + 1];
        if (cert) c.x = cert[row];
    }
    crec[4 * (int64_t)r] = rc;
    crec[4 * (int64_t)r + 1] = f0;
    crec[4 * (int64_t)r + 2] = f1;
    crec[4 * (int64_t)r + 3] = c;
    cgid[r] = (int32_t)g;
}

bool dims_ok(const PinGridDims* d) {
    return d && d->nbx > 0 && d->nby > 0 && d->nbz > 0 &&
           (int64_t)d->nbx * d->nby * d->nbz < (1ll << 31);
}

}  // namespace

extern "C" {

int pin_grid_mark(const float* positions, int64_t num_points, float resolution, const int32_t* table,
                  int64_t buffer_size, const PinGridDims* dims, uint32_t* bricks,
                  unsigned long long* counters, void* workspace, void* stream) {
    if (!dims_ok(dims) || !table || !bricks || !counters || !workspace || num_points < 0 || buffer_size <= 0 ||
        buffer_size >= (1ll << 31))
        return PIN_ERR_ARG;
    auto s = as_stream(stream);
    const int64_t nb = (int64_t)dims->nbx * dims->nby * dims->nbz;
    if (hipMemsetAsync(bricks, 0, (size_t)nb * 16, s) != hipSuccess) return PIN_ERR_HIP;
    if (hipMemsetAsync(counters, 0, 2 * sizeof(unsigned long long), s) != hipSuccess) return PIN_ERR_HIP;
    if (num_points > 0) {
        if (!positions) return PIN_ERR_ARG;
        hipLaunchKernelGGL(k_grid_mark, grid_for(num_points), dim3(kBlock), 0, s, positions, num_points, resolution,
                           table, buffer_size, *dims, bricks, counters);
    }
    const int64_t tb = std::min<int64_t>((buffer_size + 4 * kBlock - 1) / (4 * kBlock), 4096);
    hipLaunchKernelGGL(k_table_count, dim3((unsigned)tb), dim3(kBlock), 0, s, table, buffer_size, counters + 1);
    if (launch_status() != PIN_OK) return PIN_ERR_HIP;
    // brick prefix counts
    const int64_t per = (int64_t)kBlock * kScanItems;
    const int64_t np = (nb + per - 1) / per;
    uint32_t* part = (uint32_t*)workspace;  // np entries (pin_grid_workspace_bytes)
    hipLaunchKernelGGL(k_scan_partials, dim3((unsigned)np), dim3(kBlock), 0, s, bricks, nb, part);
    hipLaunchKernelGGL(k_scan_block_sums, dim3(1), dim3(1024), 0, s, part, np);
    hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)np), dim3(kBlock), 0, s, bricks, nb, part);
    return launch_status();
}

int pin_grid_fill(const float* positions, int64_t num_points, float resolution, const int32_t* table,
                  int64_t buffer_size, const PinGridDims* dims, const uint32_t* bricks, const float* records,
                  const float* features, const float* certainties, float* crec, int32_t* cgid, void* stream) {
    if (!dims_ok(dims) || !table || !bricks || !records || !crec || !cgid || num_points < 0) return PIN_ERR_ARG;
    if (num_points == 0) return PIN_OK;
    if (!positions) return PIN_ERR_ARG;
    hipLaunchKernelGGL(k_grid_fill, grid_for(num_points), dim3(kBlock), 0, as_stream(stream), positions, num_points,
                       resolution, table, buffer_size, *dims, bricks, (const float4*)records, features, certainties,
                       (float4*)crec, cgid);
    return launch_status();
}

}  // extern "C"
