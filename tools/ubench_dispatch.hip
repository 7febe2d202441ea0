// Workgroup launch-rate probe: a grid of G blocks (256 threads, L bytes of LDS) that each wait D
// microseconds (s_memrealtime, 100 MHz) and exit. Reports launch time, blocks per microsecond and
// the mean number of resident blocks (G * D / T) per (LDS, D, G).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_dispatch tools/ubench_dispatch.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

template <int LDS, int THREADS>
__global__ __launch_bounds__(THREADS) void wait_kernel(uint32_t ticks, uint32_t *sink) {
    __shared__ uint32_t pad[LDS / 4];
    pad[threadIdx.x] = threadIdx.x;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if (ticks)
        while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
    __syncthreads();
    if (pad[(threadIdx.x + 1) % THREADS] == 0xFFFFFFFFu) sink[0] = 1;
}

template <int LDS, int THREADS>
int run(uint32_t *sink, hipStream_t s) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int grids[] = {4096, 16384};
    const uint32_t us[] = {0, 1, 2, 4, 8};
    for (int g : grids)
        for (uint32_t d : us) {
            for (int w = 0; w < 3; ++w) wait_kernel<LDS, THREADS><<<g, THREADS, 0, s>>>(d * 100, sink);
            float best = 1e9f;
            for (int r = 0; r < 5; ++r) {
                CK(hipEventRecord(a, s));
                wait_kernel<LDS, THREADS><<<g, THREADS, 0, s>>>(d * 100, sink);
                CK(hipEventRecord(b, s));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                best = ms < best ? ms : best;
            }
            const double T = best * 1e3;
            printf("{\"threads\": %d, \"lds\": %d, \"grid\": %d, \"wait_us\": %u, \"launch_us\": %.2f, \"blocks_per_us\": %.1f, "
                   "\"mean_resident\": %.0f}\n",
                   THREADS, LDS, g, d, T, g / T, g * (double)d / T);
            fflush(stdout);
        }
    return 0;
}

int main() {
    uint32_t *sink;
    CK(hipMalloc(&sink, 4));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    if (run<22568, 256>(sink, s)) return 1;
    if (run<4096, 256>(sink, s)) return 1;
    if (run<45056, 512>(sink, s)) return 1;
    if (run<4096, 64>(sink, s)) return 1;
    return 0;
}
