// pin_mc.hip -- marching cubes on the device for Mesher.mc_mesh (utils/mesher.py:310-337, which
// calls skimage.measure.marching_cubes(sdf, level=0, allow_degenerate=False, mask=mc_mask)).
//
// Grid: values[nx][ny][nz] (x slowest, the reference's assign_to_bbx reshape), cube (x, y, z)
// spans grid points (x..x+1, y..y+1, z..z+1) and is processed when mask[x][y][z] is set (all
// cubes without a mask).  Triangles come from pin_mc_table.h (tools/gen_mc_table.py).  Vertices
// are shared: one per grid edge (point g, axis a) that a processed cube's triangle uses, at the
// linear crossing g + t e_a, t = (level - v_g) / (v_{g+e_a} - v_g), in index space.
//
//  pin_mc_count  k_mc_cubes   per cube: case, triangle count, flag the grid edges it uses
//                scans        edge flags -> vertex ids; triangle counts -> face offsets
//                             (device totals written to counts[2] = {vertices, faces})
//  pin_mc_emit   k_mc_verts   per flagged edge: its vertex
//                k_mc_faces   per cube: its triangles as vertex-id triples
// Workspace (pin_mc_workspace_bytes): 3 N + N_cubes int32, N_cubes int64 face offsets + rocPRIM scan scratch.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include <rocprim/device/device_scan.hpp>

#include "pin_mc_table.h"
#include "pin_slam_amd.h"

namespace {

constexpr int kMcBlock = 256;
__constant__ signed char c_tris[256][3 * PIN_MC_MAX_TRIS + 1] = PIN_MC_TRIS_INIT;
// cube edge k -> (corner offset of its lower end, axis)
__constant__ int8_t c_edge[12][4] = {{0, 0, 0, 0}, {1, 0, 0, 1}, {0, 1, 0, 0}, {0, 0, 0, 1},
                                     {0, 0, 1, 0}, {1, 0, 1, 1}, {0, 1, 1, 0}, {0, 0, 1, 1},
                                     {0, 0, 0, 2}, {1, 0, 0, 2}, {1, 1, 0, 2}, {0, 1, 0, 2}};
__constant__ int8_t c_corner[8][3] = {{0, 0, 0}, {1, 0, 0}, {1, 1, 0}, {0, 1, 0},
                                      {0, 0, 1}, {1, 0, 1}, {1, 1, 1}, {0, 1, 1}};

struct McDims {
    int64_t nx, ny, nz;
    float level;
};

__device__ __forceinline__ int64_t gidx(const McDims& d, int64_t x, int64_t y, int64_t z) {
    return (x * d.ny + y) * d.nz + z;
}

__device__ __forceinline__ int cube_case(const float* __restrict__ v, const McDims& d, int64_t x, int64_t y,
                                         int64_t z) {
    int c = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        c |= (v[gidx(d, x + c_corner[k][0], y + c_corner[k][1], z + c_corner[k][2])] < d.level) ? (1 << k) : 0;
    return c;
}

__device__ __forceinline__ void cube_of(const McDims& d, int64_t cidx, int64_t& x, int64_t& y, int64_t& z) {
    const int64_t cz = d.nz - 1, cy = d.ny - 1;
    z = cidx % cz;
    y = (cidx / cz) % cy;
    x = cidx / (cz * cy);
}

__global__ void __launch_bounds__(kMcBlock)
k_mc_cubes(const float* __restrict__ v, const uint8_t* __restrict__ mask, McDims d, int64_t ncubes,
           int32_t* __restrict__ tri_count, int32_t* __restrict__ edge_flag) {
    const int64_t c = (int64_t)blockIdx.x * kMcBlock + threadIdx.x;
    if (c >= ncubes) return;
    int64_t x, y, z;
    cube_of(d, c, x, y, z);
    int n = 0;
    if (!mask || mask[gidx(d, x, y, z)]) {
        const int cs = cube_case(v, d, x, y, z);
        const signed char* t = c_tris[cs];
        for (; n < PIN_MC_MAX_TRIS && t[3 * n] >= 0; ++n) {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int e = t[3 * n + k];
                const int64_t g = gidx(d, x + c_edge[e][0], y + c_edge[e][1], z + c_edge[e][2]);
                edge_flag[3 * g + c_edge[e][3]] = 1;   // benign race: every writer stores 1
            }
        }
    }
    tri_count[c] = n;
}

__global__ void __launch_bounds__(kMcBlock)
k_mc_verts(const float* __restrict__ v, McDims d, int64_t nedges, const int32_t* __restrict__ vid_incl,
           float* __restrict__ verts) {
    const int64_t e = (int64_t)blockIdx.x * kMcBlock + threadIdx.x;
    if (e >= nedges) return;
    const int32_t hi = vid_incl[e], lo = e ? vid_incl[e - 1] : 0;
    if (hi == lo) return;   // edge not used
    const int64_t g = e / 3;
    const int a = (int)(e - 3 * g);
    const int64_t z = g % d.nz, y = (g / d.nz) % d.ny, x = g / (d.nz * d.ny);
    const int64_t g2 = gidx(d, x + (a == 0), y + (a == 1), z + (a == 2));
    const float va = v[g], vb = v[g2];
    const float t = (d.level - va) / (vb - va);
    float p[3] = {(float)x, (float)y, (float)z};
    p[a] = p[a] + t;
    float* o = verts + 3 * (int64_t)lo;
    o[0] = p[0];
    o[1] = p[1];
    o[2] = p[2];
}

__global__ void __launch_bounds__(kMcBlock)
k_mc_faces(const float* __restrict__ v, McDims d, int64_t ncubes, const int64_t* __restrict__ tri_incl,
           const int32_t* __restrict__ vid_incl, int32_t* __restrict__ faces) {
    const int64_t c = (int64_t)blockIdx.x * kMcBlock + threadIdx.x;
    if (c >= ncubes) return;
    const int64_t end = tri_incl[c], beg = c ? tri_incl[c - 1] : 0;
    if (end == beg) return;
    int64_t x, y, z;
    cube_of(d, c, x, y, z);
    const signed char* t = c_tris[cube_case(v, d, x, y, z)];
    for (int n = 0; n < (int)(end - beg); ++n) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int e = t[3 * n + k];
            const int64_t g = gidx(d, x + c_edge[e][0], y + c_edge[e][1], z + c_edge[e][2]);
            faces[3 * (beg + n) + k] = vid_incl[3 * g + c_edge[e][3]] - 1;
        }
    }
}

__global__ void k_mc_totals(const int32_t* __restrict__ vid_incl, int64_t nedges, const int64_t* __restrict__ tri_incl,
                            int64_t ncubes, int64_t* __restrict__ counts) {
    counts[0] = nedges ? vid_incl[nedges - 1] : 0;
    counts[1] = ncubes ? tri_incl[ncubes - 1] : 0;
}

struct McLayout {
    int64_t n, ncubes, nedges;
    size_t scan_bytes;
    int32_t* edge;
    int32_t* tri;     // triangles per cube
    int64_t* tri64;   // their inclusive scan: up to 5 per cube, so int64 (2^29 cubes x 5 > 2^31)
    void* scan;
};

bool mc_dims_ok(int64_t nx, int64_t ny, int64_t nz) {
    return nx >= 2 && ny >= 2 && nz >= 2 && nx * ny * nz < (1ll << 29);   // 3 N edge ids fit int32
}

size_t mc_scan_bytes(int64_t nedges, int64_t ncubes) {
    size_t b = 0, b64 = 0;
    if (rocprim::inclusive_scan(nullptr, b, (const int32_t*)nullptr, (int32_t*)nullptr,
                                (size_t)std::max<int64_t>(nedges, 1), rocprim::plus<int32_t>()) != hipSuccess)
        return 0;
    if (rocprim::inclusive_scan(nullptr, b64, (const int32_t*)nullptr, (int64_t*)nullptr,
                                (size_t)std::max<int64_t>(ncubes, 1), rocprim::plus<int64_t>()) != hipSuccess)
        return 0;
    return std::max(b, b64);
}

McLayout mc_layout(int64_t nx, int64_t ny, int64_t nz, void* ws) {
    McLayout L;
    L.n = nx * ny * nz;
    L.ncubes = (nx - 1) * (ny - 1) * (nz - 1);
    L.nedges = 3 * L.n;
    L.scan_bytes = mc_scan_bytes(L.nedges, L.ncubes);
    char* p = (char*)ws;
    L.edge = (int32_t*)p;
    p += ((L.nedges * 4 + 255) / 256) * 256;
    L.tri = (int32_t*)p;
    p += ((L.ncubes * 4 + 255) / 256) * 256;
    L.tri64 = (int64_t*)p;
    p += ((L.ncubes * 8 + 255) / 256) * 256;
    L.scan = p;
    return L;
}

}  // namespace

extern "C" {

int64_t pin_mc_workspace_bytes(int64_t nx, int64_t ny, int64_t nz) {
    if (!mc_dims_ok(nx, ny, nz)) return -1;
    const int64_t n = nx * ny * nz, nc = (nx - 1) * (ny - 1) * (nz - 1);
    return ((3 * n * 4 + 255) / 256) * 256 + ((nc * 4 + 255) / 256) * 256 + ((nc * 8 + 255) / 256) * 256 +
           (int64_t)mc_scan_bytes(3 * n, nc) + 256;
}

int pin_mc_count(const float* values, const uint8_t* mask, int64_t nx, int64_t ny, int64_t nz, float level,
                 void* workspace, int64_t* counts, void* stream) {
    if (!mc_dims_ok(nx, ny, nz) || !values || !workspace || !counts) return PIN_ERR_ARG;
    auto s = reinterpret_cast<hipStream_t>(stream);
    McLayout L = mc_layout(nx, ny, nz, workspace);
    McDims d{nx, ny, nz, level};
    if (hipMemsetAsync(L.edge, 0, (size_t)L.nedges * 4, s) != hipSuccess) return PIN_ERR_HIP;
    hipLaunchKernelGGL(k_mc_cubes, dim3((unsigned)((L.ncubes + kMcBlock - 1) / kMcBlock)), dim3(kMcBlock), 0, s,
                       values, mask, d, L.ncubes, L.tri, L.edge);
    size_t b = L.scan_bytes;
    if (rocprim::inclusive_scan(L.scan, b, L.edge, L.edge, (size_t)L.nedges, rocprim::plus<int32_t>(), s) != hipSuccess)
        return PIN_ERR_HIP;
    b = L.scan_bytes;
    if (rocprim::inclusive_scan(L.scan, b, L.tri, L.tri64, (size_t)L.ncubes, rocprim::plus<int64_t>(), s) != hipSuccess)
        return PIN_ERR_HIP;
    hipLaunchKernelGGL(k_mc_totals, dim3(1), dim3(1), 0, s, L.edge, L.nedges, L.tri64, L.ncubes, counts);
    return hipGetLastError() == hipSuccess ? PIN_OK : PIN_ERR_HIP;
}

int pin_mc_emit(const float* values, int64_t nx, int64_t ny, int64_t nz, float level, const void* workspace,
                float* verts, int32_t* faces, void* stream) {
    if (!mc_dims_ok(nx, ny, nz) || !values || !workspace || !verts || !faces) return PIN_ERR_ARG;
    auto s = reinterpret_cast<hipStream_t>(stream);
    McLayout L = mc_layout(nx, ny, nz, const_cast<void*>(workspace));
    McDims d{nx, ny, nz, level};
    hipLaunchKernelGGL(k_mc_verts, dim3((unsigned)((L.nedges + kMcBlock - 1) / kMcBlock)), dim3(kMcBlock), 0, s,
                       values, d, L.nedges, L.edge, verts);
    hipLaunchKernelGGL(k_mc_faces, dim3((unsigned)((L.ncubes + kMcBlock - 1) / kMcBlock)), dim3(kMcBlock), 0, s,
                       values, d, L.ncubes, L.tri64, L.edge, faces);
    return hipGetLastError() == hipSuccess ? PIN_OK : PIN_ERR_HIP;
}

}  // extern "C"
