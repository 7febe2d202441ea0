// Ablation of route_kernel on the bench workloads (16 MiB batches of L-byte metrics, 4 shards).
// Every variant is an instantiation of the same kernel template (route_kernel.hpp: BLOCK threads
// per workgroup, ABL_* parts switched off). Variants are timed in interleaved rounds in ONE
// process over the same rotating set of 64 distinct batches, launched back to back from a
// hipGraph, on S concurrent streams (each stream with its own context state). A plain
// streaming-read kernel gives the achievable read rate for the same batches.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ablate_route tools/ablate_route.hip
// Run:   tools/ablate_route [line_len]
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <string>
#include <vector>

#include "../statsd-router_amd/csrc/route_host.hpp"

extern "C" {
#include "../statsd-router_amd/csrc/sr_gen.c"
}

using namespace srk;

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

__global__ __launch_bounds__(256) void read_kernel(const uint8_t *p, uint32_t n, uint32_t *sink) {
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void *)p, (short)0, (int)n, 0x00020000);
    const uint32_t T0 = blockIdx.x * 16384;
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint4 v = as_uint4(__builtin_amdgcn_raw_buffer_load_b128(rsrc, T0 + k * 4096 + threadIdx.x * 16, 0, 0));
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

constexpr int kMaxS = 4;
struct Ctx {
    DeviceState ds[kMaxS];
    std::vector<uint8_t *> batches;
    std::vector<size_t> sizes;
    sr_record *d_out[kMaxS][16];
    uint64_t *d_n;
    size_t max_lines;
    uint32_t *sink;
    hipStream_t s[kMaxS];
    hipEvent_t fork, join[kMaxS];
};

// S streams, M batches per launch (launch i routes batches i*M .. i*M+M-1 on stream i % S)
template <int BLOCK, unsigned V>
float time_variant(Ctx &c, int S, int reps, int M = 1) {
    const int B = (int)c.batches.size();
    auto launch = [&](int i) {
        const int st = i % S;
        if (V == 0xFFFFu) {
            const int k = i % B;
            hipLaunchKernelGGL(read_kernel, dim3((c.sizes[k] + 16383) / 16384), dim3(256), 0, c.s[st], c.batches[k],
                               (uint32_t)c.sizes[k], c.sink);
        } else {
            RouteParams p = c.ds[st].params();
            for (int m = 0; m < M; ++m) {
                const int k = (i * M + m) % B;
                DeviceState::add_batch(p, c.batches[k], c.sizes[k], c.d_out[st][m % 16], c.max_lines, nullptr, c.d_n + k);
            }
            launch_route<BLOCK, V>(c.ds[st], p, c.s[st]);
        }
    };
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(c.s[0], hipStreamCaptureModeGlobal));
    CK(hipEventRecord(c.fork, c.s[0]));
    for (int st = 1; st < S; ++st) CK(hipStreamWaitEvent(c.s[st], c.fork, 0));
    const int nl = V == 0xFFFFu ? B : B / M;
    for (int i = 0; i < nl; ++i) launch(i);
    for (int st = 1; st < S; ++st) {
        CK(hipEventRecord(c.join[st], c.s[st]));
        CK(hipStreamWaitEvent(c.s[0], c.join[st], 0));
    }
    CK(hipStreamEndCapture(c.s[0], &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, c.s[0]));
    CK(hipStreamSynchronize(c.s[0]));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, c.s[0]));
    for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, c.s[0]));
    CK(hipEventRecord(b, c.s[0]));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms * 1000.f / (reps * B);   // us per batch
}

int main(int argc, char **argv) {
    const int B = 64;
    const size_t batch = 16u << 20;
    uint32_t line_len = argc > 1 ? (uint32_t)atoi(argv[1]) : 64;
    CK(hipSetDevice(0));
    Ctx c;
    for (int st = 0; st < kMaxS; ++st) {
        if (c.ds[st].init(batch, 4) != 0) return 1;
        CK(hipStreamCreateWithFlags(&c.s[st], hipStreamNonBlocking));
        CK(hipEventCreateWithFlags(&c.join[st], hipEventDisableTiming));
    }
    CK(hipEventCreateWithFlags(&c.fork, hipEventDisableTiming));
    std::vector<uint8_t> host(batch);
    std::vector<size_t> lines;
    for (int b = 0; b < B; ++b) {
        size_t nd = 0, nl = 0;
        const size_t n = sr_gen_stream(0x5EED0002ull + 65537ull * b, 0, &line_len, 1, 0.0, 4095, host.data(), batch,
                                       nullptr, 0, &nd, &nl);
        uint8_t *d;
        CK(hipMalloc(&d, batch));
        CK(hipMemcpy(d, host.data(), n, hipMemcpyHostToDevice));
        c.batches.push_back(d);
        c.sizes.push_back(n);
        lines.push_back(nl);
    }
    c.max_lines = lines[0];
    for (int st = 0; st < kMaxS; ++st)
        for (int m = 0; m < 16; ++m) CK(hipMalloc(&c.d_out[st][m], c.max_lines * sizeof(sr_record)));
    CK(hipMalloc(&c.d_n, B * sizeof(uint64_t)));
    CK(hipMalloc(&c.sink, 4));

    struct Row {
        std::string name;
        float us[3];
    };
    std::vector<Row> rows;
    const int reps = 8;
    const bool quick = argc > 2 && std::string(argv[2]) == "quick";   // the parts of a 32-batch launch only
    // "alive": the shipped every-shard-alive kernel (KV_UNIFORM | KV_ALIVE, C2's) with its phases switched off
    // one at a time, 32-batch launches (per-phase VALU with tools/pmc_ablate.sh)
    const bool alive = argc > 2 && std::string(argv[2]) == "alive";
    for (int round = 0; round < 3; ++round) {
        int i = 0;
        auto put = [&](const char *name, float us) {
            if (round == 0) rows.push_back(Row{name, {0, 0, 0}});
            rows[i++].us[round] = us;
        };
        if (alive) {
            put("alive", time_variant<256, KV_ALIVE>(c, 1, reps, 32));
            put("alive_no_hash", time_variant<256, KV_ALIVE | ABL_NO_HASH>(c, 1, reps, 32));
            put("alive_no_lines", time_variant<256, KV_ALIVE | ABL_NO_LINES>(c, 1, reps, 32));
            put("alive_no_lines_no_prologue", time_variant<256, KV_ALIVE | ABL_NO_LINES | ABL_NO_PROLOGUE>(c, 1, reps, 32));
            put("alive_load_only", time_variant<256, KV_ALIVE | ABL_LOAD_ONLY | ABL_NO_LOOKBACK | ABL_NO_PROLOGUE>(c, 1, reps, 32));
            put("alive_fake_base", time_variant<256, KV_ALIVE | ABL_FAKE_BASE>(c, 1, reps, 32));
            put("read_kernel_s1", time_variant<256, 0xFFFFu>(c, 1, reps));
            continue;
        }
        if (quick) {
            put("m32", time_variant<256, ABL_NONE>(c, 1, reps, 32));
            put("m32_fake_base", time_variant<256, ABL_FAKE_BASE>(c, 1, reps, 32));
            put("m32_early_base", time_variant<256, ABL_EARLY_BASE>(c, 1, reps, 32));
            put("m32_no_mid_base", time_variant<256, ABL_NO_MID_BASE>(c, 1, reps, 32));
            put("m32_no_lookback", time_variant<256, ABL_NO_LOOKBACK>(c, 1, reps, 32));
            put("m32_no_hash", time_variant<256, ABL_NO_HASH>(c, 1, reps, 32));
            put("m32_no_prologue", time_variant<256, ABL_NO_PROLOGUE>(c, 1, reps, 32));
            put("m32_no_lines", time_variant<256, ABL_NO_LINES>(c, 1, reps, 32));
            put("m32_load_only", time_variant<256, ABL_LOAD_ONLY | ABL_NO_LOOKBACK | ABL_NO_PROLOGUE>(c, 1, reps, 32));
            put("read_kernel_s1", time_variant<256, 0xFFFFu>(c, 1, reps));
            continue;
        }
        put("b256_m16_lds_pad", time_variant<256, ABL_LDS_PAD>(c, 1, reps, 16));
        put("b256_m16_scan_serial", time_variant<256, ABL_SCAN_SERIAL>(c, 1, reps, 16));
        put("b256_m16_agent_granules", time_variant<256, ABL_AGENT_GRANULES>(c, 1, reps, 16));
        put("b256_m16_old_masks", time_variant<256, ABL_OLD_MASKS>(c, 1, reps, 16));
        put("b256_m16_old_scanner", time_variant<256, ABL_OLD_SCANNER>(c, 1, reps, 16));
        put("b256_m16_fake_base", time_variant<256, ABL_FAKE_BASE>(c, 1, reps, 16));
        put("b256_m16_fake_base_no_hash", time_variant<256, ABL_FAKE_BASE | ABL_NO_HASH>(c, 1, reps, 16));
        put("b256_m16_early_base", time_variant<256, ABL_EARLY_BASE>(c, 1, reps, 16));
        put("b256_m16_old_hash", time_variant<256, ABL_OLD_HASH>(c, 1, reps, 16));
        put("b256_m16_old_hash_no_lookback", time_variant<256, ABL_OLD_HASH | ABL_NO_LOOKBACK>(c, 1, reps, 16));
        put("b256_m16_no_hash_no_lookback", time_variant<256, ABL_NO_HASH | ABL_NO_LOOKBACK>(c, 1, reps, 16));
        put("b256_m16_no_hash_no_prologue", time_variant<256, ABL_NO_HASH | ABL_NO_PROLOGUE>(c, 1, reps, 16));
        put("b512_m16", time_variant<512, ABL_NONE>(c, 1, reps, 16));
        put("b256_m16_no_hash", time_variant<256, ABL_NO_HASH>(c, 1, reps, 16));
        put("b512_m16_no_hash", time_variant<512, ABL_NO_HASH>(c, 1, reps, 16));
        put("b256_m16", time_variant<256, ABL_NONE>(c, 1, reps, 16));
        put("b512_m16_no_lookback", time_variant<512, ABL_NO_LOOKBACK>(c, 1, reps, 16));
        put("b512_m16_no_lines", time_variant<512, ABL_NO_LINES>(c, 1, reps, 16));
        put("b512_m16_load_only", time_variant<512, ABL_LOAD_ONLY | ABL_NO_LOOKBACK | ABL_NO_PROLOGUE>(c, 1, reps, 16));
        put("b256_m16_no_lookback", time_variant<256, ABL_NO_LOOKBACK>(c, 1, reps, 16));
        put("b256_m16_no_lines", time_variant<256, ABL_NO_LINES>(c, 1, reps, 16));
        put("b256_m16_load_only", time_variant<256, ABL_LOAD_ONLY | ABL_NO_LOOKBACK | ABL_NO_PROLOGUE>(c, 1, reps, 16));
        put("b256_m1", time_variant<256, ABL_NONE>(c, 1, reps, 1));
        put("read_kernel_s1", time_variant<256, 0xFFFFu>(c, 1, reps));
        put("read_kernel_s4", time_variant<256, 0xFFFFu>(c, 4, reps));
    }
    // correctness: each product-shaped variant's line count on batch 0
    if (!quick && !alive) {
        uint64_t n = 0;
        const RouteParams p = c.ds[0].params(c.batches[0], c.sizes[0], c.d_out[0][0], c.max_lines, nullptr, c.d_n);
        launch_route<1024, ABL_NONE>(c.ds[0], p, c.s[0]);
        CK(hipMemcpyAsync(&n, c.d_n, 8, hipMemcpyDeviceToHost, c.s[0]));
        CK(hipStreamSynchronize(c.s[0]));
        fprintf(stderr, "b1024 lines %llu expected %zu\n", (unsigned long long)n, lines[0]);
        launch_route<512, ABL_NONE>(c.ds[0], p, c.s[0]);
        CK(hipMemcpyAsync(&n, c.d_n, 8, hipMemcpyDeviceToHost, c.s[0]));
        CK(hipStreamSynchronize(c.s[0]));
        fprintf(stderr, "b512 lines %llu expected %zu\n", (unsigned long long)n, lines[0]);
    }
    if (!quick && !alive) {   // multi-batch launch: every batch's line count
        std::vector<uint64_t> n(16);
        RouteParams p = c.ds[0].params();
        for (int k = 0; k < 16; ++k)
            DeviceState::add_batch(p, c.batches[k], c.sizes[k], c.d_out[0][0], c.max_lines, nullptr, c.d_n + k);
        CK(hipMemsetAsync(c.d_n, 0xFF, 16 * 8, c.s[0]));
        launch_route<512, ABL_NONE>(c.ds[0], p, c.s[0]);
        CK(hipMemcpyAsync(n.data(), c.d_n, 16 * 8, hipMemcpyDeviceToHost, c.s[0]));
        CK(hipStreamSynchronize(c.s[0]));
        int bad = 0;
        for (int k = 0; k < 16; ++k) bad += n[k] != lines[k];
        fprintf(stderr, "b512 m16: %d of 16 batch counts wrong\n", bad);
    }
    printf("{\"line_len\": %u, \"batch_bytes\": %zu, \"us_per_batch\": {", line_len, batch);
    for (size_t r = 0; r < rows.size(); ++r) {
        float best = 1e9f;
        for (int k = 0; k < 3; ++k) best = fminf(best, rows[r].us[k]);
        printf("%s\"%s\": [%.2f, %.0f]", r ? ", " : "", rows[r].name.c_str(), best, batch / (best * 1e-6) / 1e9);
    }
    printf("}}\n");
    return 0;
}
