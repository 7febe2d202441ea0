// hbm_read.hip — the measured streaming-read ceiling bench.py reports beside the route kernel's
// roofline fraction ("also report a measured streaming-read ceiling"). A read-only
// kernel over the same resident batches: 16 B per lane per load, 8 loads in flight per lane, a
// grid-stride over the buffer, one XOR per block stored so the loads cannot be dropped.
// Measurement tooling, not the product (built into tools/hbm/libsr_hbm.so).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {
constexpr int kBlock = 256, kUnroll = 8;
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(kBlock) void hbm_read_kernel(const v4u32 *__restrict__ p, uint64_t n16,
                                                          uint32_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock * kUnroll;
    uint32_t acc = 0;
    for (uint64_t base = (uint64_t)blockIdx.x * kBlock * kUnroll + threadIdx.x; base < n16; base += stride) {
        v4u32 v[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const uint64_t i = base + (uint64_t)u * kBlock;
            v[u] = i < n16 ? __builtin_nontemporal_load(&p[i]) : (v4u32){0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    __shared__ uint32_t s[kBlock];
    s[threadIdx.x] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t a = 0;
        for (int i = 0; i < kBlock; ++i) a ^= s[i];
        out[blockIdx.x] = a;
    }
}
// One 16 KiB tile per workgroup, the route kernel's access pattern (lane = 64 contiguous bytes, four
// 16-B loads at +0/16/32/48) or the coalesced one (load k: lanes on consecutive 16 B of quarter k).
template <bool kCoalesced>
__global__ __launch_bounds__(kBlock) void tile_read_kernel(const v4u32 *__restrict__ p, uint32_t *__restrict__ out) {
    const uint64_t t16 = (uint64_t)blockIdx.x * 1024;   // 16-B units per tile
    v4u32 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        v[k] = kCoalesced ? p[t16 + (uint64_t)k * 256 + threadIdx.x] : p[t16 + (uint64_t)threadIdx.x * 4 + k];
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    if (acc == 0x9E3779B9u) out[blockIdx.x] = acc;   // keeps the loads
}
}  // namespace

// mode 0: the streaming kernel above; 1: one tile per workgroup, route pattern; 2: the same, coalesced
extern "C" int sr_hbm_read_mode(const void *d, size_t nbytes, uint32_t *d_out, uint32_t blocks, void *stream,
                                int mode) {
    if (mode == 0) {
        hipLaunchKernelGGL(hbm_read_kernel, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream, (const v4u32 *)d,
                           (uint64_t)(nbytes / 16), d_out);
    } else {
        const uint32_t tiles = (uint32_t)(nbytes / 16384);
        if (mode == 1)
            hipLaunchKernelGGL(tile_read_kernel<false>, dim3(tiles), dim3(kBlock), 0, (hipStream_t)stream,
                               (const v4u32 *)d, d_out);
        else
            hipLaunchKernelGGL(tile_read_kernel<true>, dim3(tiles), dim3(kBlock), 0, (hipStream_t)stream,
                               (const v4u32 *)d, d_out);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int sr_hbm_read(const void *d, size_t nbytes, uint32_t *d_out, uint32_t blocks, void *stream) {
    if (!d || !d_out || blocks == 0 || (nbytes & 15)) return -1;
    hipLaunchKernelGGL(hbm_read_kernel, dim3(blocks), dim3(kBlock), 0, (hipStream_t)stream, (const v4u32 *)d,
                       (uint64_t)(nbytes / 16), d_out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
