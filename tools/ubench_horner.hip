// Microbenchmark: VALU cost of one sdbm step h = h*65599 + (int8)c on gfx950, by formulation.
// Each thread runs R rounds over 64 register-resident bytes; reports bytes/s chip-wide.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_horner tools/ubench_horner.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int R = 256;
constexpr uint64_t K = 65599;

__device__ __forceinline__ uint64_t step_c(uint64_t h, uint32_t b) {
    return h * K + (uint64_t)(int64_t)(int8_t)b;
}

__device__ __forceinline__ uint64_t step_shift(uint64_t h, uint32_t b) {
    uint64_t c = (uint64_t)(int64_t)(int8_t)b, t;
    // t = (h << 6) + c ; t = (h << 16) + t ; h = t - h
    asm volatile("v_lshl_add_u64 %0, %1, 6, %2" : "=v"(t) : "v"(h), "v"(c));
    asm volatile("v_lshl_add_u64 %0, %1, 16, %2" : "=v"(t) : "v"(h), "v"(t));
    return t - h;
}

__device__ __forceinline__ uint64_t step_shift_nc(uint64_t h, uint32_t b) {
    // (h << 16) + (h << 6) - h + c written plainly; let the compiler pick
    const int64_t c = (int8_t)b;
    return (h << 16) + (h << 6) - h + (uint64_t)c;
}

// two bytes per step: w = c0*K + c1 (24-bit signed mad, exact), h = h*K^2 + w
__device__ __forceinline__ uint64_t step_pair(uint64_t h, uint32_t b0, uint32_t b1) {
    const int32_t w = __builtin_amdgcn_sbfe(b0, 0, 8) * (int32_t)K + __builtin_amdgcn_sbfe(b1, 0, 8);
    return h * (K * K) + (uint64_t)(int64_t)w;
}

__device__ __forceinline__ uint64_t step_dword(uint64_t h, uint32_t x) {
    const int32_t c0 = (int8_t)(x & 0xFFu), c1 = (int8_t)((x >> 8) & 0xFFu);
    const int32_t c2 = (int8_t)((x >> 16) & 0xFFu), c3 = (int8_t)(x >> 24);
    const int32_t t = c0 * (int32_t)K + c1;
    const int32_t u = c2 * (int32_t)K + c3;
    const uint64_t d = (uint64_t)((int64_t)t * 0x7E0F81) + (uint64_t)(int64_t)u + ((uint64_t)(uint32_t)t << 32);
    return h * (K * K * K * K) + d;
}

template <int V>
__global__ void kern(const uint32_t *in, uint64_t *out) {
    uint32_t d[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) d[i] = in[(threadIdx.x * 16 + i) & 4095] ^ blockIdx.x;
    uint64_t h = threadIdx.x;
    for (int r = 0; r < R; ++r) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t x = d[i] + r;
            if (V == 0) { h = step_c(h, x); h = step_c(h, x >> 8); h = step_c(h, x >> 16); h = step_c(h, x >> 24); }
            if (V == 1) { h = step_shift(h, x); h = step_shift(h, x >> 8); h = step_shift(h, x >> 16); h = step_shift(h, x >> 24); }
            if (V == 2) { h = step_shift_nc(h, x & 0xFF); h = step_shift_nc(h, (x >> 8) & 0xFF); h = step_shift_nc(h, (x >> 16) & 0xFF); h = step_shift_nc(h, x >> 24); }
            if (V == 3) { h = step_pair(h, x, x >> 8); h = step_pair(h, x >> 16, x >> 24); }
            if (V == 4) { h = step_dword(h, x); }
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = h;
}

template <int V>
double run(const uint32_t *in, uint64_t *out, int blocks) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    kern<V><<<blocks, 256>>>(in, out);
    hipEventRecord(a);
    for (int i = 0; i < 5; ++i) kern<V><<<blocks, 256>>>(in, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double bytes = 5.0 * blocks * 256.0 * R * 64.0;
    return bytes / (ms * 1e-3) / 1e12;
}

int main() {
    uint32_t *in;
    uint64_t *out;
    const int blocks = 256 * 16;
    hipMalloc(&in, 4096 * 4);
    hipMalloc(&out, (size_t)blocks * 256 * 8);
    hipMemset(in, 0x5A, 4096 * 4);
    printf("{\"horner_TBps\": {\"mad_u64_compiler\": %.2f, \"lshl_add_u64_asm\": %.2f, "
           "\"shift_plain\": %.2f, \"pair_k2\": %.2f, \"dword_k4\": %.2f}}\n",
           run<0>(in, out, blocks), run<1>(in, out, blocks), run<2>(in, out, blocks), run<3>(in, out, blocks), run<4>(in, out, blocks));
    return 0;
}
