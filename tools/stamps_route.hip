// Diagnostic timeline of route_kernel (ABL_STAMPS build): s_memrealtime (100 MHz) at phase
// boundaries in every workgroup, for back-to-back launches on 16 distinct batches.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/stamps_route tools/stamps_route.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
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

static double med(std::vector<double> v) {
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

// one launch over all L batches (the product's multi-batch mode): per-phase medians over every
// workgroup of the launch, plus the launch span
static bool seg_layout = false, chunk_layout = false;

template <int BLOCK>
void run_many(DeviceState &ds, std::vector<uint8_t *> &batches, std::vector<size_t> &sizes, sr_record *d_out,
              size_t max_lines, uint64_t *d_n, uint64_t *d_dbg, hipStream_t s, uint32_t line_len) {
    const int L = (int)batches.size();
    const uint32_t T = BLOCK * kLaneBytes;
    uint32_t total = 0;
    for (int i = 0; i < L; ++i) total += (uint32_t)((sizes[i] + T - 1) / T);
    std::vector<uint64_t> h((size_t)total * 16);
    auto launch = [&]() {
        RouteParams p = ds.params();
        for (int i = 0; i < L; ++i)
            DeviceState::add_batch(p, batches[i], sizes[i], d_out + (size_t)i * max_lines, max_lines, nullptr, d_n + i);
        p.dbg = d_dbg;
        if (chunk_layout) launch_route<BLOCK, ABL_STAMPS | KV_CHUNKS | KV_ALIVE>(ds, p, s);
        else if (seg_layout) launch_route<BLOCK, ABL_STAMPS | KV_SEGMENTS | KV_ALIVE>(ds, p, s);
        else launch_route<BLOCK, ABL_STAMPS | KV_ALIVE>(ds, p, s);
    };
    for (int w = 0; w < 3; ++w) launch();
    CK(hipStreamSynchronize(s));
    CK(hipMemsetAsync(d_dbg, 0, (size_t)16 * 4096 * 16 * 8, s));
    CK(hipStreamSynchronize(s));
    launch();
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(h.data(), d_dbg, h.size() * 8, hipMemcpyDeviceToHost));
    {   // record-base chain: tile order per batch (16 batches -> XCD classes j % 8, j and j + 8 share one)
        std::vector<uint32_t> nt(L);
        for (int i = 0; i < L; ++i) nt[i] = (uint32_t)((sizes[i] + T - 1) / T);
        std::vector<std::vector<uint32_t>> order(L);   // per batch: block g of each tile
        for (uint32_t g = 0; g < total; ++g) {
            const uint32_t cls = g & 7, ci = g >> 3;
            const int j = ci < nt[cls] ? (int)cls : (int)cls + 8;
            const uint32_t t = ci < nt[cls] ? ci : ci - nt[cls];
            if (j < L && t < nt[j]) {
                if (order[j].size() <= t) order[j].resize(t + 1, ~0u);
                order[j][t] = g;
            }
        }
        std::vector<double> late, lag;
        size_t waited = 0, n = 0;
        for (int j = 0; j < L; ++j) {
            uint64_t m = 0;
            for (size_t t = 0; t < order[j].size(); ++t) {
                const uint64_t *d = h.data() + (size_t)order[j][t] * 16;
                ++n;
                if (d[3]) {
                    ++waited;
                    late.push_back(((double)m - (double)d[3]) * 0.01);
                    lag.push_back(((double)d[7] - (double)std::max(m, d[3])) * 0.01);
                }
                m = std::max(m, d[1]);
            }
        }
        std::sort(late.begin(), late.end());
        std::sort(lag.begin(), lag.end());
        auto pc = [](std::vector<double> &v, double q) { return v.empty() ? 0.0 : v[(size_t)(q * (v.size() - 1))]; };
        printf("{\"base_chain\": {\"tiles\": %zu, \"polled\": %zu, \"pred_count_late_us\": [%.2f, %.2f, %.2f, %.2f], "
               "\"lag_after_counts_us\": [%.2f, %.2f, %.2f, %.2f]}}\n",
               n, waited, pc(late, 0.1), pc(late, 0.5), pc(late, 0.9), pc(late, 0.99), pc(lag, 0.1), pc(lag, 0.5),
               pc(lag, 0.9), pc(lag, 0.99));
    }
    {   // raw per-tile dump for offline analysis: entry, stamp0, end, exit, hw_id, xcc
        FILE *f = fopen("gpurun_out/stamps_raw.bin", "wb");
        if (f) {
            for (uint32_t t = 0; t < total; ++t) {
                const uint64_t *d = h.data() + (size_t)t * 16;
                const uint64_t r[12] = {d[8], d[0], d[6], d[9], d[10], d[11], d[3], d[7], d[1], d[13], d[12], d[4]};
                fwrite(r, 8, 12, f);
            }
            fclose(f);
        }
    }
    {   // scanner poll rounds (batch 0 and 8): round-trip percentiles and round count
        std::vector<uint64_t> sc(16 * 4096);
        CK(hipMemcpy(sc.data(), d_dbg + 300000, 16 * 4096 * 8, hipMemcpyDeviceToHost));
        std::vector<double> rt;
        int nr = 0;
        for (int b = 0; b < 16; ++b)
            for (int r = 0; r < 2048; ++r) {
                const uint64_t a = sc[b * 4096 + 2 * r], z = sc[b * 4096 + 2 * r + 1];
                if (a && z) rt.push_back((double)(z - a) * 0.01), ++nr;
            }
        std::sort(rt.begin(), rt.end());
        if (!rt.empty())
            printf("{\"scanner_poll_rt_us\": [%.2f, %.2f, %.2f, %.2f], \"rounds_per_batch\": %.1f}\n", rt[rt.size() / 10],
                   rt[rt.size() / 2], rt[rt.size() * 9 / 10], rt[rt.size() * 99 / 100], nr / 16.0);
    }
    std::vector<double> ph[8], ph3b;
    uint64_t s0 = ~0ull, e1 = 0;
    {   // residency: tiles alive over the launch (start stamp 0 .. end stamp 6), in 1 us bins
        std::vector<std::pair<uint64_t, uint64_t>> iv;
        for (uint32_t b = 0; b < total; ++b) {
            const uint64_t *d = h.data() + (size_t)b * 16;
            if (d[8] && d[9]) iv.push_back({d[8], d[9]});   // kernel entry .. after arrive
        }
        uint64_t a = ~0ull, z = 0;
        double busy = 0;
        for (auto &x : iv) a = std::min(a, x.first), z = std::max(z, x.second), busy += (double)(x.second - x.first);
        const int nb = (int)((z - a) / 100) + 1;
        std::vector<double> occ(nb, 0.0), starts(nb, 0.0);
        for (auto &x : iv) {
            starts[(x.first - a) / 100] += 1;
            for (uint64_t t = x.first; t < x.second; t += 10) occ[(t - a) / 100] += 0.1;
        }
        printf("{\"residency\": {\"span_us\": %.2f, \"mean_resident_tiles\": %.1f, \"per_us\": [", (z - a) * 0.01,
               busy / (double)(z - a));
        for (int i = 0; i < nb; ++i) printf("%s[%.0f, %.0f]", i ? ", " : "", occ[i], starts[i]);
        printf("]}}\n");
    }
    for (uint32_t b = 0; b < total; ++b) {
        const uint64_t *d = h.data() + (size_t)b * 16;
        if (!d[0]) continue;
        s0 = std::min(s0, d[0]);
        e1 = std::max(e1, d[6]);
        const double u = 0.01;
        ph[0].push_back((d[1] - d[0]) * u);
        ph[1].push_back((d[2] - d[1]) * u);
        if (d[3]) ph[2].push_back((d[7] - d[3]) * u);   // base wait (tid 0, first record), when polled
        ph[3].push_back((d[4] - d[2]) * u);
        ph[4].push_back((d[5] - d[4]) * u);
        if (d[14]) ph3b.push_back((d[14] - d[4]) * u);   // segment pre-pass
        ph[5].push_back((d[6] - d[0]) * u);
        ph[6].push_back((d[0] - d[8]) * u);   // entry: epoch, batch lookup, load issue
        ph[7].push_back((d[9] - d[8]) * u);   // entry .. after arrive
    }
    {
        std::vector<double> w = ph[2];
        if (w.empty()) w.push_back(0.0);
        std::sort(w.begin(), w.end());
        printf("{\"base_wait_us_percentiles\": {\"p10\": %.2f, \"p50\": %.2f, \"p90\": %.2f, \"p99\": %.2f}}\n",
               w[w.size() / 10], w[w.size() / 2], w[w.size() * 9 / 10], w[w.size() * 99 / 100]);
    }
    printf("{\"mode\": \"%d batches per launch\", \"block\": %d, \"line_len\": %u, \"tiles\": %u, \"span_us\": %.2f, "
           "\"median_us\": {\"load\": %.2f, \"masks_scan\": %.2f, \"base_wait\": %.2f, \"to_staged\": %.2f, "
           "\"hash_records\": %.2f, \"of_which_prepass\": %.2f, \"lifetime\": %.2f, \"entry\": %.2f, \"entry_to_exit\": %.2f}}\n",
           L, BLOCK, line_len, total, (e1 - s0) * 0.01, med(ph[0]), med(ph[1]), med(ph[2]), med(ph[3]), med(ph[4]),
           med(ph3b), med(ph[5]), med(ph[6]), med(ph[7]));
}

int main(int argc, char **argv) {
    const int L = 16;
    const size_t batch = 16u << 20;
    // argv: line length (0 = the C5 mix 64/256/1024), shards, "seg" / "chunks" for those layouts
    uint32_t line_len = argc > 1 ? (uint32_t)atoi(argv[1]) : 64;
    const uint32_t nds = argc > 2 ? (uint32_t)atoi(argv[2]) : 4;
    seg_layout = argc > 3 && !strcmp(argv[3], "seg");
    chunk_layout = argc > 3 && !strcmp(argv[3], "chunks");   // route_chunk_kernel: stamps 0 loads in, 1 after
                                                             // the count barrier, 2 Suf done, 4 slots done,
                                                             // 5 records, 6 before the look-back, 9 exit
    uint32_t mix[3] = {64, 256, 1024};
    const uint32_t *lens = line_len ? &line_len : mix;
    const uint32_t nlens = line_len ? 1u : 3u;
    CK(hipSetDevice(0));
    DeviceState ds;
    if (ds.init(batch, nds) != 0) return 1;
    std::vector<uint8_t> host(batch);
    std::vector<uint8_t *> batches;
    std::vector<size_t> sizes;
    size_t nl = 0, nd = 0;
    for (int b = 0; b < L; ++b) {
        const size_t n = sr_gen_stream(0x5EED0002ull + 65537ull * b, 0, lens, nlens, 0.0, 4095, host.data(), batch,
                                       nullptr, 0, &nd, &nl);
        uint8_t *d;
        CK(hipMalloc(&d, batch));
        CK(hipMemcpy(d, host.data(), n, hipMemcpyHostToDevice));
        batches.push_back(d);
        sizes.push_back(n);
    }
    sr_record *d_out;
    uint64_t *d_n, *d_dbg;
    CK(hipMalloc(&d_out, (size_t)L * nl * sizeof(sr_record)));
    CK(hipMalloc(&d_n, 8 * L));
    CK(hipMalloc(&d_dbg, (size_t)L * 4096 * 16 * 8));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    run_many<256>(ds, batches, sizes, d_out, nl, d_n, d_dbg, s, line_len);
    return 0;
}
