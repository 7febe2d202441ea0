// exchange.hpp — the multi-GPU exchange of owner packs over RCCL (xGMI), for C hosts
// (include/sr_route.h: sr_comm_*, sr_exchange_sizes, sr_exchange_data).
//
// Shard s is owned by GPU s % G. Every GPU routes its own datagram batches and packs the valid
// lines by owner (sr_pack_by_owner / sr_pack_many_by_owner: owner chunks back to back, the
// records' offsets relative to their owner's chunk, split sizes {lines, bytes} per owner). The
// exchange is two collective calls per route launch:
//   sizes: an all-to-all of the split sizes, then ONE copy of the sent and received sizes to the
//          host (the launch's only host round trip: the receive buffers are sized from it);
//   data : grouped ncclSend / ncclRecv of every peer's chunk of lines and of records, then the
//          rebase of the received records' offsets into the receive buffer (source p's bytes land
//          after those of sources 0 .. p-1, so its offsets move by their total).
// RCCL is opened with dlopen at sr_comm_open: libsr_route.so does not depend on it otherwise, and a
// process that already holds RCCL (e.g. PyTorch's) shares that copy.
#pragma once

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "regroup_kernel.hpp"

namespace srk {

// the RCCL entry points used here (rccl.h types spelled out: the header is not needed to build)
enum : int { kNcclUint8 = 1, kNcclUint64 = 5 };
struct RcclApi {
    void *so = nullptr;
    int (*get_unique_id)(void *id) = nullptr;
    void *comm_init_rank = nullptr;   // InitRankFn (below): the unique id travels by value
    int (*comm_destroy)(void *comm) = nullptr;
    int (*all_to_all)(const void *, void *, size_t, int, void *, hipStream_t) = nullptr;
    int (*send)(const void *, size_t, int, int, void *, hipStream_t) = nullptr;
    int (*recv)(void *, size_t, int, int, void *, hipStream_t) = nullptr;
    int (*group_start)() = nullptr;
    int (*group_end)() = nullptr;
};

struct CommId {
    char b[128];
};
using InitRankFn = int (*)(void **, int, CommId, int);

inline RcclApi *rccl_api() {
    static RcclApi api;
    static bool tried = false;
    if (tried) return api.so ? &api : nullptr;
    tried = true;
    void *so = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);   // already in the process
    if (!so) so = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!so) so = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!so) return nullptr;
    api.get_unique_id = (int (*)(void *))dlsym(so, "ncclGetUniqueId");
    api.comm_init_rank = dlsym(so, "ncclCommInitRank");
    api.comm_destroy = (int (*)(void *))dlsym(so, "ncclCommDestroy");
    api.all_to_all = (int (*)(const void *, void *, size_t, int, void *, hipStream_t))dlsym(so, "ncclAllToAll");
    api.send = (int (*)(const void *, size_t, int, int, void *, hipStream_t))dlsym(so, "ncclSend");
    api.recv = (int (*)(void *, size_t, int, int, void *, hipStream_t))dlsym(so, "ncclRecv");
    api.group_start = (int (*)())dlsym(so, "ncclGroupStart");
    api.group_end = (int (*)())dlsym(so, "ncclGroupEnd");
    if (!api.get_unique_id || !api.comm_init_rank || !api.comm_destroy || !api.all_to_all || !api.send ||
        !api.recv || !api.group_start || !api.group_end)
        return nullptr;
    api.so = so;
    return &api;
}

// Received records from source p (lines [line0[p], line0[p+1])) move by byte0[p].
struct RebaseArgs {
    uint32_t sources;
    uint32_t n_lines;
    uint32_t line0[kMaxOwners + 1];
    uint32_t byte0[kMaxOwners];
};

__global__ __launch_bounds__(256) void exchange_rebase_kernel(sr_record *recs, RebaseArgs a) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= a.n_lines) return;
    uint32_t lo = 0, hi = a.sources;   // the source: the last p with line0[p] <= i
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a.line0[mid] <= i) lo = mid;
        else hi = mid;
    }
    recs[i].offset += a.byte0[lo];
}

}  // namespace srk
