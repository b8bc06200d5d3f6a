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
//   crec[r]    = 16-byte record {x, y, z, bits(id)} of the r-th occupied cell in brick order
//   cfeat[r]   = its 8 features, ccert[r] = its certainty (inference copies, optional)
//   cgid[r]    = global point index of that record
// Brick order keeps the candidates of one query within a few 128-B lines: a surface brick
// holds ~16 occupied cells = 256 B of records.
// The bricks of a 1M-point surface map are ~2 MB: L2-resident on every XCD, so the
// probe phase costs L1/L2 hits and only real candidates touch HBM (one line each).
#include <hip/hip_runtime.h>

#include <climits>
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

// grid-stride: each thread marks its points' bits; the own-cell count is reduced per block
// and added with one atomic per block (a per-wave atomic on one address serialises)
__device__ __forceinline__ void block_count_add(unsigned long long c, unsigned long long* __restrict__ counter) {
    __shared__ unsigned long long red[kBlock / 64];
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < kBlock / 64; ++w) t += red[w];
        if (t) atomicAdd(counter, t);
    }
}

__global__ void __launch_bounds__(kBlock)
k_grid_mark(const float* __restrict__ pos, int64_t M, float res, const int32_t* __restrict__ table, int64_t B,
            PinGridDims d, uint32_t* __restrict__ bricks, unsigned long long* __restrict__ marked) {
    unsigned long long c = 0;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < M; g += stride) {
        int64_t brick;
        int bit;
        if (own_cell(pos, g, res, B, table, d, brick, bit)) {
            atomicOr(bricks + 4 * brick + (bit >> 5), 1u << (bit & 31));
            ++c;
        }
    }
    block_count_add(c, marked);
}

__global__ void __launch_bounds__(kBlock)
k_table_count(const int32_t* __restrict__ table, int64_t B, unsigned long long* __restrict__ count) {
    unsigned long long c = 0;
    constexpr int U = 4;  // independent 16-B loads in flight per thread
    const int64_t nvec = B / 4;
    const int4* __restrict__ t4 = (const int4*)table;
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    for (; i + (U - 1) * stride < nvec; i += U * stride) {
        int4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = t4[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) c += (v[u].x >= 0) + (v[u].y >= 0) + (v[u].z >= 0) + (v[u].w >= 0);
    }
    for (; i < nvec; i += stride) {
        const int4 v = t4[i];
        c += (v.x >= 0) + (v.y >= 0) + (v.z >= 0) + (v.w >= 0);
    }
    if (blockIdx.x == 0 && threadIdx.x < (B & 3)) c += table[nvec * 4 + threadIdx.x] >= 0;
    block_count_add(c, count);
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
            float4* __restrict__ cfeat, float* __restrict__ ccert, int32_t* __restrict__ cgid) {
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
    const int64_t row = id & kIdMask;
    crec[r] = rc;
    cgid[r] = (int32_t)g;
    if (cfeat) {
        float4 f0 = make_float4(0.f, 0.f, 0.f, 0.f), f1 = f0;
        if (id != -1 && feat) {
            f0 = ((const float4*)feat)[2 * row];
            f1 = ((const float4*)feat)[2 * row + 1];
        }
        cfeat[2 * (int64_t)r] = f0;
        cfeat[2 * (int64_t)r + 1] = f1;
    }
    if (ccert) ccert[r] = (id != -1 && cert) ? cert[row] : 0.f;
}

bool dims_ok(const PinGridDims* d) {
    return d && d->nbx > 0 && d->nby > 0 && d->nbz > 0 &&
           (int64_t)d->nbx * d->nby * d->nbz < (1ll << 31);
}

// cell-index bounding box of the points: per-thread min/max over a grid-stride loop, wave and
// block reductions, then one 64-bit atomic per block and component
__global__ void k_bounds_init(long long* out) {
    if (threadIdx.x < 3) out[threadIdx.x] = LLONG_MAX;
    else if (threadIdx.x < 6) out[threadIdx.x] = LLONG_MIN;
}

__global__ void __launch_bounds__(kBlock)
k_cell_bounds(const float* __restrict__ pos, int64_t M, float res, long long* __restrict__ out) {
    long long lo[3] = {LLONG_MAX, LLONG_MAX, LLONG_MAX}, hi[3] = {LLONG_MIN, LLONG_MIN, LLONG_MIN};
    const int64_t stride = (int64_t)gridDim.x * kBlock;
    for (int64_t g = (int64_t)blockIdx.x * kBlock + threadIdx.x; g < M; g += stride) {
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const long long c = (long long)floorf(pos[3 * g + a] / res);
            lo[a] = c < lo[a] ? c : lo[a];
            hi[a] = c > hi[a] ? c : hi[a];
        }
    }
    __shared__ long long red[kBlock / 64][6];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        for (int off = 32; off > 0; off >>= 1) {
            const long long l = __shfl_xor(lo[a], off), h = __shfl_xor(hi[a], off);
            lo[a] = l < lo[a] ? l : lo[a];
            hi[a] = h > hi[a] ? h : hi[a];
        }
        if ((threadIdx.x & 63) == 0) {
            red[threadIdx.x >> 6][a] = lo[a];
            red[threadIdx.x >> 6][3 + a] = hi[a];
        }
    }
    __syncthreads();
    if (threadIdx.x < 6) {
        long long v = red[0][threadIdx.x];
        for (int w = 1; w < kBlock / 64; ++w) {
            const long long t = red[w][threadIdx.x];
            v = threadIdx.x < 3 ? (t < v ? t : v) : (t > v ? t : v);
        }
        if (threadIdx.x < 3) atomicMin(out + threadIdx.x, v);
        else atomicMax(out + threadIdx.x, v);
    }
}

}  // namespace

extern "C" {

int pin_cell_bounds(const float* positions, int64_t num_points, float resolution, int64_t* out, void* stream) {
    if (!out || num_points < 0 || (num_points > 0 && !positions) || !(resolution > 0.f)) return PIN_ERR_ARG;
    auto s = as_stream(stream);
    hipLaunchKernelGGL(k_bounds_init, dim3(1), dim3(64), 0, s, (long long*)out);
    if (num_points > 0) {
        const int64_t nblk = std::min<int64_t>((num_points + kBlock - 1) / kBlock, 2048);
        hipLaunchKernelGGL(k_cell_bounds, dim3((unsigned)nblk), dim3(kBlock), 0, s, positions, num_points, resolution,
                           (long long*)out);
    }
    return launch_status();
}


int pin_grid_mark_ex(const float* positions, int64_t num_points, float resolution, const int32_t* table,
                     int64_t buffer_size, const PinGridDims* dims, uint32_t* bricks, unsigned long long* counters,
                     void* workspace, int32_t flags, void* stream) {
    if (flags & ~PIN_GRID_TABLE_TRUSTED) return PIN_ERR_ARG;
    if (!dims_ok(dims) || !table || !bricks || !counters || !workspace || num_points < 0 || buffer_size <= 0 ||
        buffer_size >= (1ll << 31))
        return PIN_ERR_ARG;
    auto s = as_stream(stream);
    const int64_t nb = (int64_t)dims->nbx * dims->nby * dims->nbz;
    if (hipMemsetAsync(bricks, 0, (size_t)nb * 16, s) != hipSuccess) return PIN_ERR_HIP;
    if (hipMemsetAsync(counters, 0, 2 * sizeof(unsigned long long), s) != hipSuccess) return PIN_ERR_HIP;
    if (num_points > 0) {
        if (!positions) return PIN_ERR_ARG;
        const int64_t mb = std::min<int64_t>((num_points + kBlock - 1) / kBlock, 4096);
        hipLaunchKernelGGL(k_grid_mark, dim3((unsigned)mb), dim3(kBlock), 0, s, positions, num_points, resolution,
                           table, buffer_size, *dims, bricks, counters);
    }
    if (flags & PIN_GRID_TABLE_TRUSTED) {
        // the caller vouches that every occupied slot holds a point of its own cell: occupied =
        // marked, no pass over the table
        if (hipMemcpyAsync(counters + 1, counters, sizeof(unsigned long long), hipMemcpyDeviceToDevice, s) !=
            hipSuccess)
            return PIN_ERR_HIP;
    } else {
        const int64_t tb = std::min<int64_t>(std::max<int64_t>((buffer_size / 4 + kBlock - 1) / kBlock, 1), 2048);
        hipLaunchKernelGGL(k_table_count, dim3((unsigned)tb), dim3(kBlock), 0, s, table, buffer_size, counters + 1);
    }
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

int pin_grid_mark(const float* positions, int64_t num_points, float resolution, const int32_t* table,
                  int64_t buffer_size, const PinGridDims* dims, uint32_t* bricks,
                  unsigned long long* counters, void* workspace, void* stream) {
    return pin_grid_mark_ex(positions, num_points, resolution, table, buffer_size, dims, bricks, counters, workspace,
                            0, stream);
}

int pin_grid_fill(const float* positions, int64_t num_points, float resolution, const int32_t* table,
                  int64_t buffer_size, const PinGridDims* dims, const uint32_t* bricks, const float* records,
                  const float* features, const float* certainties, float* crec, float* cfeat, float* ccert,
                  int32_t* cgid, void* stream) {
    if (!dims_ok(dims) || !table || !bricks || !records || !crec || !cgid || num_points < 0) return PIN_ERR_ARG;
    if (num_points == 0) return PIN_OK;
    if (!positions) return PIN_ERR_ARG;
    hipLaunchKernelGGL(k_grid_fill, grid_for(num_points), dim3(kBlock), 0, as_stream(stream), positions, num_points,
                       resolution, table, buffer_size, *dims, bricks, (const float4*)records, features, certainties,
                       (float4*)crec, (float4*)cfeat, ccert, cgid);
    return launch_status();
}

}  // extern "C"
