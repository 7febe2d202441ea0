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
#include <errno.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <mutex>

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

inline RcclApi *rccl_load(RcclApi &api) {
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

inline RcclApi *rccl_api() {   // loaded once per process (data threads may race here)
    static RcclApi api;
    static RcclApi *loaded = nullptr;
    static std::once_flag once;
    std::call_once(once, [] { loaded = rccl_load(api); });
    return loaded;
}

// Received records from source p (lines [line0[p], line0[p+1])) move by byte0[p].
struct RebaseArgs {
    uint32_t sources;
    uint32_t n_lines;
    uint32_t first;     // the first line that moves: sources before it land at byte 0 (source 0 always)
    uint32_t line0[kMaxOwners + 1];
    uint32_t byte0[kMaxOwners];
};

// The exchange plan (sr_exchange_plan): per peer the pack's chunk sent to it and where its chunk
// lands. Chunks are owner-major in the pack (sr_pack_many_by_owner) and source-major in the receive
// buffers, so both sides are exclusive prefix sums of the split sizes.
inline int exchange_plan(int world, int rank, const uint64_t *sent, const uint64_t *received,
                         sr_exchange_peer *peers, uint64_t totals[4]) {
    if (world < 1 || world > kMaxOwners || rank < 0 || rank >= world || !sent || !received || !peers)
        return -EINVAL;
    uint64_t s_l = 0, s_b = 0, r_l = 0, r_b = 0;
    for (int q = 0; q < world; ++q) {
        sr_exchange_peer &e = peers[q];
        e.send_line0 = s_l, e.send_lines = sent[2 * q];
        e.send_byte0 = s_b, e.send_bytes = sent[2 * q + 1];
        e.recv_line0 = r_l, e.recv_lines = received[2 * q];
        e.recv_byte0 = r_b, e.recv_bytes = received[2 * q + 1];
        s_l += e.send_lines, s_b += e.send_bytes, r_l += e.recv_lines, r_b += e.recv_bytes;
        if (s_l < e.send_lines || s_b < e.send_bytes || r_l < e.recv_lines || r_b < e.recv_bytes) return -EINVAL;
    }
    // the own chunk is copied, so both sides of the all-to-all must agree on it
    if (peers[rank].send_lines != peers[rank].recv_lines || peers[rank].send_bytes != peers[rank].recv_bytes)
        return -EINVAL;
    if (r_b > 0xFFFFFFFFull || r_l > 0xFFFFFFFFull) return -EINVAL;   // record offsets are u32
    if (totals) totals[0] = s_l, totals[1] = s_b, totals[2] = r_l, totals[3] = r_b;
    return 0;
}

inline int rebase_args(const sr_exchange_peer *peers, int world, RebaseArgs &a) {
    if (world < 1 || world > kMaxOwners) return -EINVAL;
    memset(&a, 0, sizeof(a));
    uint64_t l = 0;
    for (int q = 0; q < world; ++q) {
        if (peers[q].recv_line0 != l || peers[q].recv_byte0 > 0xFFFFFFFFull) return -EINVAL;
        a.line0[q] = (uint32_t)l;
        a.byte0[q] = (uint32_t)peers[q].recv_byte0;
        l += peers[q].recv_lines;
    }
    if (l > 0xFFFFFFFFull) return -EINVAL;
    a.sources = (uint32_t)world;
    a.n_lines = (uint32_t)l;
    a.first = a.n_lines;
    for (int q = 0; q < world; ++q)
        if (a.byte0[q]) {
            a.first = a.line0[q];
            break;
        }
    a.line0[world] = (uint32_t)l;
    return 0;
}

// One exchange over a transport (sr_exchange_run): the plan, the peers' sends and receives in one
// group (rank order; bytes then records; zero sizes skipped on both sides, since my send size to q
// is q's receive size from me), the own chunk, then the rebase.
inline int exchange_run(const sr_transport &t, int world, int rank, const uint64_t *sent, const uint64_t *received,
                        const uint8_t *packed, const sr_record *packed_recs, uint8_t *recv_bytes,
                        sr_record *recv_recs, bool own_in_place = false) {
    if (!t.group_start || !t.group_end || !t.send || !t.recv || !t.copy || !t.rebase) return -EINVAL;
    sr_exchange_peer peers[kMaxOwners];
    uint64_t tot[4];
    int rc = exchange_plan(world, rank, sent, received, peers, tot);
    if (rc) return rc;
    if ((tot[1] && !packed) || (tot[0] && !packed_recs) || (tot[3] && !recv_bytes) || (tot[2] && !recv_recs))
        return -EINVAL;
    if ((rc = t.group_start(t.user))) return rc;
    // Every operation is posted even after one fails, so that the peers' matching operations can
    // complete and no peer waits forever inside the group; the first error is returned. A transport
    // error still leaves the communicator unusable: the caller destroys it (sr_comm_close).
    int bad = 0;
    auto post = [&bad](int r) {
        if (r && !bad) bad = r;
    };
    for (int q = 0; q < world; ++q) {
        if (q == rank) continue;
        const sr_exchange_peer &e = peers[q];
        if (e.send_bytes) post(t.send(t.user, packed + e.send_byte0, e.send_bytes, q, 0));
        if (e.recv_bytes) post(t.recv(t.user, recv_bytes + e.recv_byte0, e.recv_bytes, q, 0));
        if (e.send_lines) post(t.send(t.user, packed_recs + e.send_line0, e.send_lines * sizeof(sr_record), q, 1));
        if (e.recv_lines) post(t.recv(t.user, recv_recs + e.recv_line0, e.recv_lines * sizeof(sr_record), q, 1));
    }
    rc = t.group_end(t.user);   // always closed, also after a failed post
    if (bad) return bad;
    if (rc) return rc;
    const sr_exchange_peer &own = peers[rank];   // (own_in_place: the pack wrote it there)
    if (!own_in_place && own.send_bytes &&
        (rc = t.copy(t.user, recv_bytes + own.recv_byte0, packed + own.send_byte0, own.send_bytes)))
        return rc;
    if (!own_in_place && own.send_lines &&
        (rc = t.copy(t.user, recv_recs + own.recv_line0, packed_recs + own.send_line0, own.send_lines * sizeof(sr_record))))
        return rc;
    return tot[2] ? t.rebase(t.user, recv_recs, peers, world, tot[2]) : 0;
}

// The split sizes to the host in one launch (sr_exchange_sizes): sent and received {lines, bytes}
// (u64 [world][2] each) into mapped, coherent pinned memory, then a sequence word after a system-scope
// fence, which the host polls; no copy launches and no blocking stream synchronisation on the launch's
// one host round trip. recv == nullptr (one rank, no collective): the received sizes are the sent ones,
// also written to d_recv. One workgroup of 256 threads, w2 = 2 * world <= 128.
__global__ __launch_bounds__(256) void sizes_publish_kernel(const uint64_t *sent, const uint64_t *recv,
                                                             uint64_t *d_recv, uint64_t *h, uint32_t w2, uint64_t seq) {
    const uint32_t t = threadIdx.x;
    if (t < w2) {
        const uint64_t v = sent[t];
        h[t] = v;
        if (!recv) d_recv[t] = v;
    } else if (t >= 128 && t - 128 < w2) {
        h[w2 + t - 128] = (recv ? recv : sent)[t - 128];
    }
    __threadfence_system();
    __syncthreads();
    if (t == 0) *(volatile uint64_t *)(h + 2 * w2) = seq;
}

__global__ __launch_bounds__(256) void exchange_rebase_kernel(sr_record *recs, RebaseArgs a) {
    const uint32_t i = a.first + blockIdx.x * 256u + threadIdx.x;
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
