// sr_route.hip — MI355X (gfx950) implementation of statsd-router's per-datagram hot path.
//
// Reference path (hulu/statsd-router, /root/reference):
//   udp_read_cb        sr-main.c:149-191  framing + newline tokeniser + length gate 5 < L < 1450
//   process_data_line  sr-main.c:137-147  ':' presence -> INVALID_FORMAT
//   hash               sr-main.c:120-134  sdbm over the name (signed char, u64 wrap)
//   find_downstream    sr-main.c:86-117   hash-seeded partial Fisher-Yates probe over alive shards
//
// Input: a batch of framed datagrams laid back to back in HBM. Every framed datagram ends in
// '\n' (host framing, sr_frame_datagram), so the lines of the batch are its '\n'-terminated
// pieces and datagram boundaries are irrelevant to the GPU. Output: one 8-byte sr_record per
// line, in input order (include/sr_route.h).
//
// One kernel, one pass over the bytes (design: DESIGN.md §3):
//   * 16 KiB tiles, one 256-thread workgroup each; tile ids come from an atomic ticket so the
//     decoupled look-back below can never wait on a workgroup that has not started.
//   * Tile bytes: coalesced 1 KiB-per-wave-instruction buffer loads -> LDS; each lane then owns
//     64 contiguous bytes.
//   * Per lane: '\n' and ':' bitmasks (SWAR), and the unmasked sdbm Horner value Q of its 64
//     bytes. The name hash of a line [s, c) is a difference of prefix values,
//         h = P(c-1) - P(s-1) * K^(c-s)   (mod 2^64, K = 65599),
//     where P is the Horner prefix over the tile; P comes from a wave + workgroup scan of the
//     lane values with the constant multiplier K^64, stored per 16-byte piece in LDS.
//   * Line numbering: a workgroup scan of per-lane '\n' counts gives tile-local line indices;
//     the tile's first record index comes from a decoupled look-back over per-tile counts
//     (8-byte {epoch, flag, count} granules, agent-scope relaxed atomics: the data is the flag).
//   * A line that starts in an earlier tile (at most one per tile) is finished from a short
//     backward re-read of the previous tile's tail by wave 0.
//   * Shard pick: h % N through a precomputed 64-bit magic reciprocal when every shard is alive;
//     otherwise the reference's probe with a 16-entry register overlay of the permutation
//     (a dead shard is probed at most once per line). Lines needing more than 16 dead probes are
//     deferred to probe_wide_kernel, which runs the probe on a full LDS permutation.
// No MFMA: this is HBM-bound byte work (VALU + LDS).

#include <hip/hip_runtime.h>

#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/sr_route.h"

namespace {

constexpr int kBlock = 256;                  // threads per workgroup (4 waves)
constexpr int kLaneBytes = 64;               // bytes per lane
constexpr int kTile = kBlock * kLaneBytes;   // 16 KiB per tile
constexpr int kPieces = kTile / 16;          // 16-byte pieces per tile
constexpr int kWindow = 2048;                // tile-local lines staged in LDS per round
constexpr int kOverlay = 16;                 // register overlay entries of the probe
constexpr int kNone = 0x7FFF;                // "no colon" marker (int16 in linfo)
constexpr uint32_t kFlagAgg = 1u, kFlagIncl = 2u;
constexpr uint16_t kRoutePending = 0xFFFCu;  // internal: resolved by probe_wide_kernel
constexpr uint64_t K = 65599ull;             // sdbm multiplier: (h<<6)+(h<<16)-h (sr-main.c:131)
constexpr int kPowTable = 4097;              // K^0 .. K^4096

constexpr uint64_t ipow(uint64_t b, unsigned e) {
    uint64_t r = 1;
    while (e) {
        if (e & 1) r *= b;
        b *= b;
        e >>= 1;
    }
    return r;
}
constexpr uint64_t inv_odd(uint64_t a) {  // a^-1 mod 2^64 for odd a (Newton)
    uint64_t x = a;
    for (int i = 0; i < 6; ++i) x *= 2 - a * x;
    return x;
}
constexpr uint64_t kK16 = ipow(K, 16), kK32 = ipow(K, 32), kK48 = ipow(K, 48), kK64 = ipow(K, 64);
constexpr uint64_t kK4096 = ipow(K, 4096);
constexpr uint64_t kKinv = inv_odd(K);
static_assert(K * kKinv == 1ull, "K inverse");

struct Magic {          // exact n / d for 64-bit n (Granlund-Montgomery, round-up variant)
    uint64_t m;
    uint32_t shift;
    uint32_t kind;      // 0: q = n >> shift; 1: q = mulhi >> shift; 2: add-indicator form
};

struct PendingLine {
    uint32_t rec;
    uint32_t pad;
    uint64_t hash;
};

// Per-context device control block. Zeroed once at sr_open; the kernel keeps it consistent:
// the last workgroup to finish resets ticket/done and bumps epoch.
struct Control {
    uint32_t ticket;
    uint32_t done;
    uint32_t epoch;
    uint32_t pending;
};

struct RouteParams {
    const uint8_t *bytes;
    uint32_t nbytes;
    uint32_t ntiles;
    sr_record *recs;
    uint64_t *hashes;        // may be null
    uint64_t *n_out;         // device: total line count
    uint32_t max_records;
    uint32_t nds;            // number of downstreams
    uint32_t dead;           // dead downstreams in the alive snapshot
    uint32_t pending_cap;
    Magic magic_n;           // for h % nds (fast path)
    const uint64_t *alive;   // bitmap
    const Magic *magic;      // [0..nds], index i -> divisor i
    const uint64_t *kpow;    // K^0..K^4096
    Control *ctl;
    uint64_t *status;        // per-tile look-back granules
    PendingLine *pending;
};

__constant__ uint64_t c_kpow16[17];   // K^0 .. K^16
__constant__ uint64_t c_kinv[64];     // K^-0 .. K^-63
__constant__ uint64_t c_klane[64];    // K^(64*l)

// ---------------------------------------------------------------------------------------
// Scalar helpers
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t sdbm_step(uint64_t h, uint32_t byte) {
    // sr-main.c:131: h = (h << 6) + (h << 16) - h + c, with c a *signed* char (sr-main.c:122)
    const int64_t c = (int8_t)byte;
    return (h << 16) + (h << 6) - h + (uint64_t)c;
}

__device__ __forceinline__ uint64_t sdbm_dword(uint64_t h, uint32_t x) {
    h = sdbm_step(h, x & 0xFFu);
    h = sdbm_step(h, (x >> 8) & 0xFFu);
    h = sdbm_step(h, (x >> 16) & 0xFFu);
    return sdbm_step(h, x >> 24);
}

// 4-bit mask of the bytes of x equal to the byte replicated in pat (exact SWAR test).
__device__ __forceinline__ uint32_t eq_mask4(uint32_t x, uint32_t pat) {
    const uint32_t t = x ^ pat;
    const uint32_t z = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
    return (((z >> 7) * 0x00204081u) >> 21) & 0xFu;
}

// 16 bytes at `off`; bytes at or past `n` read as 0. Only the one piece that straddles the end
// of the batch takes the byte-wise path (buffer range checks are not byte-exact for dwordx4).
__device__ __forceinline__ uint4 load16(__amdgpu_buffer_rsrc_t rsrc, uint32_t off, uint32_t n) {
    if (off + 16u <= n) {
        const auto r = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
        return make_uint4(r[0], r[1], r[2], r[3]);
    }
    uint64_t lo = 0, hi = 0;
    for (uint32_t i = 0; i < 16u && off + i < n; ++i) {
        const uint64_t b = __builtin_amdgcn_raw_buffer_load_b8(rsrc, off + i, 0, 0);
        if (i < 8) lo |= b << (8 * i);
        else hi |= b << (8 * (i - 8));
    }
    return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

__device__ __forceinline__ uint64_t div_magic(uint64_t n, const Magic &mg) {
    if (mg.kind == 0) return n >> mg.shift;
    const uint64_t t = __umul64hi(mg.m, n);
    if (mg.kind == 1) return t >> mg.shift;
    return (((n - t) >> 1) + t) >> mg.shift;
}

__device__ __forceinline__ uint32_t mod_magic(uint64_t n, const Magic &mg, uint32_t d) {
    return (uint32_t)(n - div_magic(n, mg) * (uint64_t)d);
}

__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int d) {
    const uint32_t lo = __shfl_up((uint32_t)v, d, 64);
    const uint32_t hi = __shfl_up((uint32_t)(v >> 32), d, 64);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int d) {
    const uint32_t lo = __shfl_xor((uint32_t)v, d, 64);
    const uint32_t hi = __shfl_xor((uint32_t)(v >> 32), d, 64);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += shfl_xor64(v, d);
    return v;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, lane);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

// Segmented "line state" scan element: [63:32] newline count, [31] lane range holds a '\n',
// [15:0] first ':' of the line open at the right end of the range (tile position, kNone = none).
// combine(f, g) for f left of g: counts add; if g holds a '\n' its state wins, else the open
// line continues from f and its first colon is the earlier one.
__device__ __forceinline__ uint64_t seg_combine(uint64_t f, uint64_t g) {
    const uint64_t cnt = (f & 0xFFFFFFFF00000000ull) + (g & 0xFFFFFFFF00000000ull);
    uint32_t lo;
    if ((uint32_t)g & 0x80000000u) {
        lo = (uint32_t)g;
    } else {
        const uint32_t fc = (uint32_t)f & 0xFFFFu, gc = (uint32_t)g & 0xFFFFu;
        lo = ((uint32_t)f & 0xFFFF0000u) | (fc < gc ? fc : gc);
    }
    return cnt | lo;
}

__device__ __forceinline__ uint64_t mk_status(uint32_t epoch, uint32_t flag, uint32_t value) {
    return ((uint64_t)(epoch & 0x3FFFFFFFu) << 34) | ((uint64_t)flag << 32) | value;
}

__device__ __forceinline__ bool alive_bit(const uint64_t *alive, uint32_t k) {
    return (alive[k >> 6] >> (k & 63)) & 1ull;
}

// find_downstream (sr-main.c:86-117) for one line. Returns the shard, SR_ROUTE_ALL_DEAD, or
// kRoutePending if more than kOverlay dead shards had to be probed.
__device__ uint32_t probe_shard(uint64_t h, const RouteParams &p) {
    const uint32_t n = p.nds;
    if (p.dead >= n) return SR_ROUTE_ALL_DEAD;            // includes N == 0
    if (p.dead == 0) return mod_magic(h, p.magic_n, n);   // every shard alive: j = h % N
    // ds_index[] is the identity plus an overlay of (position -> value) writes, newest last.
    uint32_t ov[kOverlay];   // (pos << 16) | value
    int nov = 0;
#pragma unroll
    for (int e = 0; e < kOverlay; ++e) ov[e] = 0xFFFFFFFFu;
    for (uint32_t i = n; i > 0; --i) {
        const Magic mg = p.magic[i];
        const uint32_t j = mod_magic(h, mg, i);                      // :98
        uint32_t k = j;                                              // :99
#pragma unroll
        for (int e = 0; e < kOverlay; ++e)
            if ((ov[e] >> 16) == j) k = ov[e] & 0xFFFFu;
        if (alive_bit(p.alive, k)) return k;                         // :101-104
        if (j != i - 1) {                                            // :108-111
            uint32_t v = i - 1;
#pragma unroll
            for (int e = 0; e < kOverlay; ++e)
                if ((ov[e] >> 16) == i - 1) v = ov[e] & 0xFFFFu;
            if (nov == kOverlay) return kRoutePending;
#pragma unroll
            for (int e = 0; e < kOverlay; ++e)
                if (e == nov) ov[e] = (j << 16) | v;
            ++nov;
        }
        h = (h * 7 + 5) / 3;                                         // :113
    }
    return SR_ROUTE_ALL_DEAD;                                        // :115-116
}

// ---------------------------------------------------------------------------------------
// The route kernel
// ---------------------------------------------------------------------------------------
struct __align__(16) Smem {
    uint4 tile[kPieces];             // 16 KiB: the tile's bytes
    uint64_t pstate[kPieces];        // P(16p - 1) for every 16-byte piece p (tile frame, P(-1)=0)
    uint32_t linfo[kWindow + 1];     // per line: e | (uint16)c << 16; slot 0 = previous line
    uint64_t wave_seg[4];
    uint64_t wave_hash[4];
    uint64_t h_pre, hc_pre;          // straddling line: Horner of [s_pre, 0) and [s_pre, c_pre)
    int32_t s_pre, c_pre;            // tile-relative start / first colon (c_pre: kNone if none)
    uint32_t tile_id, epoch, base, count;
};

// P(x) in the tile frame for -1 <= x < kTile: Horner of tile bytes [0, x].
__device__ __forceinline__ uint64_t prefix_at(const Smem &sm, int x) {
    if (x < 0) return 0;
    const int pc = x >> 4, r = x & 15;
    const uint4 v = sm.tile[pc];
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint64_t t = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int keep = r + 1 - 4 * k;   // bytes of dword k at or before x
        const uint32_t m = keep >= 4 ? 0xFFFFFFFFu : (keep <= 0 ? 0u : ((1u << (8 * keep)) - 1u));
        t = sdbm_dword(t, w[k] & m);
    }
    // t = Horner(bytes[16pc .. x]) * K^(15 - r); undo the trailing zeros with K^-1.
    return sm.pstate[pc] * c_kpow16[r + 1] + t * c_kinv[15 - r];
}

__global__ __launch_bounds__(kBlock) void route_kernel(RouteParams p) {
    __shared__ Smem sm;
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;

    if (tid == 0) {
        sm.tile_id = atomicAdd(&p.ctl->ticket, 1u);
        sm.epoch = __hip_atomic_load(&p.ctl->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // Coalesced tile load: wave instruction k of thread tid covers bytes k*4096 + tid*16.
    // Out-of-range bytes read as 0 (buffer descriptor range check), never as '\n' or ':'.
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void *)p.bytes, (short)0, (int)p.nbytes, 0x00020000);
    __syncthreads();
    const uint32_t t = sm.tile_id;
    const uint32_t epoch = sm.epoch;
    const int64_t T0 = (int64_t)t * kTile;
    {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = load16(rsrc, (uint32_t)T0 + k * 4096 + tid * 16, p.nbytes);
#pragma unroll
        for (int k = 0; k < 4; ++k) sm.tile[k * 256 + tid] = v[k];
    }

    // ---- wave 0: the line that straddles into this tile (starts before T0) ----------------
    if (wave == 0) {
        int64_t s_abs = 0;
        if (t > 0) {
            int64_t hi = T0, found = -1;
            for (;;) {
                const int64_t lo = hi - 1024 > 0 ? hi - 1024 : 0;
                const int64_t a = lo + lane * 16;
                uint32_t nl16 = 0;
                if (a < hi) {
                    const auto r = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (uint32_t)a, 0, 0);
#pragma unroll
                    for (int k = 0; k < 4; ++k) nl16 |= eq_mask4(r[k], 0x0A0A0A0Au) << (4 * k);
                }
                const uint64_t m = __ballot(nl16 != 0);
                if (m) {
                    const int L = 63 - __builtin_clzll(m);
                    const int64_t last = a + 31 - __builtin_clz(nl16 | 1u);  // valid on lane L
                    found = (int64_t)readlane64((uint64_t)last, L);
                    break;
                }
                if (lo == 0) break;
                hi = lo;
            }
            s_abs = found + 1;
        }
        const int32_t s_pre = (int32_t)(s_abs - T0);
        uint64_t h_pre = 0, hc_pre = 0;
        int32_t c_pre = kNone;
        if (s_pre < 0 && -s_pre <= (int)SR_MAX_LINE_LENGTH - 1) {
            // Horner over [s_abs, T0) in aligned 32-byte chunks, one per lane.
            const int64_t A = s_abs & ~31ll;
            const int nch = (int)((T0 - A) >> 5);   // <= 47
            uint64_t q = 0;
            uint32_t cm = 0;
            uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            if (lane < nch) {
                const int64_t a = A + 32 * lane;
                const auto r0 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (uint32_t)a, 0, 0);
                const auto r1 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (uint32_t)a + 16, 0, 0);
                w[0] = r0[0]; w[1] = r0[1]; w[2] = r0[2]; w[3] = r0[3];
                w[4] = r1[0]; w[5] = r1[1]; w[6] = r1[2]; w[7] = r1[3];
                // zero the bytes before s_abs (leading zeros do not change a Horner value)
                const int64_t skip = s_abs - a;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const int64_t sk = skip - 4 * k;
                    const uint32_t m = sk <= 0 ? 0xFFFFFFFFu : (sk >= 4 ? 0u : ~((1u << (8 * sk)) - 1u));
                    w[k] &= m;
                    cm |= (eq_mask4(w[k], 0x3A3A3A3Au)) << (4 * k);
                    q = sdbm_dword(q, w[k]);
                }
            }
            const uint64_t wgt = lane < nch ? p.kpow[32 * (nch - 1 - lane)] : 0;
            h_pre = wave_sum64(q * wgt);
            const uint64_t cl = __ballot(cm != 0);
            if (cl) {
                const int lc = __builtin_ctzll(cl);
                const int mpos = (int)__builtin_amdgcn_readlane(cm ? __builtin_ctz(cm) : 0, lc);
                c_pre = (int32_t)(A + 32 * lc + mpos - T0);
                // lanes before lc contribute whole chunks; lane lc its bytes before the colon
                uint64_t qc = 0;
                if (lane == lc) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        const int keep = mpos - 4 * k;
                        const uint32_t m = keep >= 4 ? 0xFFFFFFFFu : (keep <= 0 ? 0u : ((1u << (8 * keep)) - 1u));
                        qc = sdbm_dword(qc, w[k] & m);
                    }
                } else if (lane < lc) {
                    qc = q * p.kpow[32 * (lc - lane)];
                }
                hc_pre = wave_sum64(qc) * c_kinv[32 - mpos];
            }
        }
        if (lane == 0) {
            sm.s_pre = s_pre;
            sm.c_pre = c_pre;
            sm.h_pre = h_pre;
            sm.hc_pre = hc_pre;
        }
    }
    __syncthreads();

    // ---- per lane: 64 contiguous bytes -------------------------------------------------------
    const int o = tid * kLaneBytes;   // tile position of the lane's first byte
    uint64_t nlm = 0, clm = 0;        // bit i: byte o+i is '\n' / ':'
    uint64_t q = 0, q16 = 0, q32 = 0, q48 = 0;
#pragma unroll
    for (int pc = 0; pc < 4; ++pc) {
        const uint4 v = sm.tile[tid * 4 + pc];
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int sh = 16 * pc + 4 * k;
            nlm |= (uint64_t)eq_mask4(w[k], 0x0A0A0A0Au) << sh;
            clm |= (uint64_t)eq_mask4(w[k], 0x3A3A3A3Au) << sh;
            q = sdbm_dword(q, w[k]);
        }
        if (pc == 0) q16 = q;
        if (pc == 1) q32 = q;
        if (pc == 2) q48 = q;
    }
    const int ncnt = __popcll(nlm);
    // segmented line state of the lane
    uint64_t seg;
    {
        uint32_t fc;
        if (nlm) {
            const int lastb = 63 - __clzll(nlm);
            const uint64_t after = lastb == 63 ? 0ull : (clm & (~0ull << (lastb + 1)));
            fc = after ? (uint32_t)(o + __ffsll((long long)after) - 1) : (uint32_t)kNone;
            seg = ((uint64_t)ncnt << 32) | 0x80000000u | fc;
        } else {
            fc = clm ? (uint32_t)(o + __ffsll((long long)clm) - 1) : (uint32_t)kNone;
            seg = fc;
        }
    }
    // wave inclusive scans: seg (line state) and q (Horner, multiplier K^64 per lane)
    uint64_t sseg = seg, shash = q;
    {
        uint64_t mul = kK64;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t a = shfl_up64(sseg, d);
            const uint64_t b = shfl_up64(shash, d);
            if (lane >= d) {
                sseg = seg_combine(a, sseg);
                shash = b * mul + shash;
            }
            mul *= mul;
        }
    }
    if (lane == 63) {
        sm.wave_seg[wave] = sseg;
        sm.wave_hash[wave] = shash;
    }
    __syncthreads();
    // exclusive values for this lane (tile frame, carry-in empty)
    uint64_t eseg = shfl_up64(sseg, 1);
    uint64_t ehash = shfl_up64(shash, 1);
    if (lane == 0) {
        eseg = (uint64_t)kNone;   // empty range: count 0, no '\n', no colon
        ehash = 0;
    }
    {
        uint64_t cseg = (uint64_t)kNone, chash = 0;   // carry of the waves before this one
        for (int w2 = 0; w2 < wave; ++w2) {
            cseg = seg_combine(cseg, sm.wave_seg[w2]);
            chash = chash * kK4096 + sm.wave_hash[w2];
        }
        eseg = seg_combine(cseg, eseg);
        ehash = chash * c_klane[lane] + ehash;
    }
    const uint32_t tile_count = (uint32_t)((seg_combine(seg_combine(seg_combine(sm.wave_seg[0],
                                    sm.wave_seg[1]), sm.wave_seg[2]), sm.wave_seg[3])) >> 32);
    // piece prefix values P(16p - 1)
    sm.pstate[tid * 4 + 0] = ehash;
    sm.pstate[tid * 4 + 1] = ehash * kK16 + q16;
    sm.pstate[tid * 4 + 2] = ehash * kK32 + q32;
    sm.pstate[tid * 4 + 3] = ehash * kK48 + q48;

    // publish this tile's aggregate early (tile 0: its inclusive prefix)
    if (tid == 0) {
        const uint64_t st = mk_status(epoch, t == 0 ? kFlagIncl : kFlagAgg, tile_count);
        __hip_atomic_store(&p.status[t], st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    // ---- decoupled look-back (wave 0) -------------------------------------------------------
    if (wave == 0) {
        uint64_t acc = 0;
        if (t > 0) {
            int64_t pred = (int64_t)t - 1;
            for (;;) {
                const int64_t idx = pred - lane;
                uint64_t st = mk_status(epoch, kFlagIncl, 0);   // before tile 0: inclusive 0
                if (idx >= 0)
                    st = __hip_atomic_load(&p.status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint32_t flag = (uint32_t)(st >> 32) & 3u;
                const bool valid = (uint32_t)(st >> 34) == (epoch & 0x3FFFFFFFu) && flag != 0;
                const uint64_t vm = __ballot(valid);
                const uint64_t im = __ballot(valid && flag == kFlagIncl);
                const int first_invalid = ~vm ? __builtin_ctzll(~vm) : 64;
                const int first_incl = im ? __builtin_ctzll(im) : 64;
                if (first_incl < first_invalid) {
                    acc += wave_sum64(lane <= first_incl ? (st & 0xFFFFFFFFull) : 0);
                    break;
                }
                if (first_invalid > 0) {
                    acc += wave_sum64(lane < first_invalid ? (st & 0xFFFFFFFFull) : 0);
                    pred -= first_invalid;
                } else {
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            if (lane == 0) {
                const uint64_t st = mk_status(epoch, kFlagIncl, (uint32_t)(acc + tile_count));
                __hip_atomic_store(&p.status[t], st, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (lane == 0) {
            sm.base = (uint32_t)acc;
            sm.count = tile_count;
            if (t == p.ntiles - 1) *p.n_out = acc + tile_count;
        }
    }
    __syncthreads();
    const uint32_t base = sm.base;
    const int s_pre = sm.s_pre;
    const int c_pre = sm.c_pre;

    // ---- per line: windows of kWindow tile-local lines ------------------------------------
    const int lane_first = (int)(eseg >> 32);               // tile-local index of lane's 1st line
    const bool open_has_nl = (uint32_t)eseg & 0x80000000u;  // a '\n' earlier in the tile
    int open_fc = (int)((uint32_t)eseg & 0xFFFFu);          // first ':' of the open line
    if (!open_has_nl && c_pre != kNone) open_fc = c_pre;    // straddling line: colon before T0
    if (tid == 0) sm.linfo[0] = 0;
    for (int wbase = 0; wbase < (int)tile_count; wbase += kWindow) {
        // (1) stage (e, c) of the lane's lines that fall into this window
        if (nlm && lane_first + ncnt > wbase && lane_first < wbase + kWindow) {
            uint64_t m = nlm;
            int idx = lane_first;
            int prevb = -1;
            while (m) {
                const int b = __builtin_ctzll(m);
                m &= m - 1;
                int c;
                if (prevb < 0 && open_fc != kNone) {
                    c = open_fc;
                } else {
                    const uint64_t below = b == 0 ? 0ull : (~0ull >> (64 - b));
                    const uint64_t above = ~0ull << (prevb + 1);
                    const uint64_t cm = clm & below & above;
                    c = cm ? o + __builtin_ctzll(cm) : kNone;
                }
                if (idx >= wbase && idx < wbase + kWindow)
                    sm.linfo[idx - wbase + 1] = (uint32_t)(o + b) | ((uint32_t)(uint16_t)(int16_t)c << 16);
                ++idx;
                prevb = b;
            }
        }
        __syncthreads();
        // (2) one thread per line
        const int nwin = min(kWindow, (int)tile_count - wbase);
        for (int jj = tid; jj < nwin; jj += kBlock) {
            const int j = wbase + jj;
            const uint32_t li = sm.linfo[jj + 1];
            const int e = (int)(li & 0xFFFFu);
            const int c = (int)(int16_t)(uint16_t)(li >> 16);
            const int s = (j == 0) ? s_pre : (int)(sm.linfo[jj] & 0xFFFFu) + 1;
            const int64_t len = (int64_t)e - s + 1;
            uint32_t route;
            uint64_t h = 0;
            if (len < (int)SR_MIN_LINE_LENGTH || len > (int)SR_MAX_LINE_LENGTH) {   // sr-main.c:180
                route = SR_ROUTE_INVALID_LENGTH;
            } else if (c == kNone || c > e) {                                        // sr-main.c:140
                route = SR_ROUTE_INVALID_FORMAT;
            } else {
                if (j == 0) {
                    h = c < 0 ? sm.hc_pre : sm.h_pre * p.kpow[c] + prefix_at(sm, c - 1);
                } else {
                    h = prefix_at(sm, c - 1) - prefix_at(sm, s - 1) * p.kpow[c - s];
                }
                route = probe_shard(h, p);
            }
            const uint32_t rec = base + (uint32_t)j;
            if (rec < p.max_records) {
                if (route == kRoutePending) {
                    const uint32_t slot = atomicAdd(&p.ctl->pending, 1u);
                    if (slot < p.pending_cap) p.pending[slot] = PendingLine{rec, 0u, h};
                }
                sr_record r;
                r.offset = (uint32_t)(T0 + s);
                r.length = len > 0xFFFF ? (uint16_t)0xFFFF : (uint16_t)len;
                r.route = (uint16_t)route;
                p.recs[rec] = r;
                if (p.hashes) p.hashes[rec] = h;
            }
        }
        __syncthreads();
        if (tid == 0) sm.linfo[0] = sm.linfo[nwin];
        __syncthreads();
    }

    // ---- last workgroup out resets the ticket and advances the epoch -----------------------
    if (tid == 0) {
        const uint32_t d = atomicAdd(&p.ctl->done, 1u);
        if (d == p.ntiles - 1) {
            __hip_atomic_store(&p.ctl->ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&p.ctl->done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&p.ctl->epoch, epoch + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// Lines whose probe met more than kOverlay dead shards: run find_downstream (sr-main.c:86-117)
// literally on a permutation array held in LDS (N <= 65533 -> <= 128 KiB), one line at a time
// per workgroup. After each line the touched entries are restored by replaying the probe.
__global__ __launch_bounds__(64) void probe_wide_kernel(RouteParams p) {
    extern __shared__ uint16_t ds_index[];
    const uint32_t n = p.nds;
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) ds_index[i] = (uint16_t)i;
    __syncthreads();
    const uint32_t np = min(__hip_atomic_load(&p.ctl->pending, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                            p.pending_cap);
    if (threadIdx.x != 0) return;
    for (uint32_t x = blockIdx.x; x < np; x += gridDim.x) {
        const PendingLine pl = p.pending[x];
        uint64_t h = pl.hash;
        uint32_t route = SR_ROUTE_ALL_DEAD, steps = 0;
        for (uint32_t i = n; i > 0; --i) {
            const uint32_t j = mod_magic(h, p.magic[i], i);
            const uint32_t k = ds_index[j];
            ++steps;
            if (alive_bit(p.alive, k)) { route = k; break; }
            if (j != i - 1) {
                ds_index[j] = ds_index[i - 1];
                ds_index[i - 1] = (uint16_t)k;
            }
            h = (h * 7 + 5) / 3;
        }
        p.recs[pl.rec].route = (uint16_t)route;
        // restore the identity on every touched position
        h = pl.hash;
        for (uint32_t i = n; i > 0 && steps > 0; --i, --steps) {
            const uint32_t j = mod_magic(h, p.magic[i], i);
            ds_index[j] = (uint16_t)j;
            ds_index[i - 1] = (uint16_t)(i - 1);
            h = (h * 7 + 5) / 3;
        }
    }
}

// ---------------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------------
Magic make_magic(uint64_t d) {
    Magic mg{0, 0, 0};
    if (d == 0) return mg;
    const int fl = 63 - __builtin_clzll(d);
    if ((d & (d - 1)) == 0) {
        mg.shift = (uint32_t)fl;
        mg.kind = 0;
        return mg;
    }
    const unsigned __int128 num = (unsigned __int128)1 << (64 + fl);
    uint64_t pm = (uint64_t)(num / d);
    const uint64_t rem = (uint64_t)(num % d);
    const uint64_t e = d - rem;
    if (e < (1ull << fl)) {
        mg.kind = 1;
    } else {
        pm += pm;
        const uint64_t twice = rem + rem;
        if (twice >= d || twice < rem) pm += 1;
        mg.kind = 2;
    }
    mg.m = pm + 1;
    mg.shift = (uint32_t)fl;
    return mg;
}

uint64_t host_div(uint64_t n, const Magic &mg) {
    if (mg.kind == 0) return n >> mg.shift;
    const uint64_t t = (uint64_t)(((unsigned __int128)mg.m * n) >> 64);
    if (mg.kind == 1) return t >> mg.shift;
    return (((n - t) >> 1) + t) >> mg.shift;
}

bool tables_uploaded[64];

}  // namespace

struct sr_ctx {
    int device;
    hipStream_t own_stream;
    hipStream_t stream;
    size_t max_batch;
    uint32_t nds;
    uint32_t nwords;
    uint32_t dead;
    uint32_t max_tiles;
    uint64_t *h_alive;
    // device buffers
    uint8_t *d_in;
    sr_record *d_out;
    size_t d_out_cap;
    uint64_t *d_hash;
    size_t d_hash_cap;
    uint64_t *d_count;
    uint64_t *d_alive;
    Magic *d_magic;
    Magic magic_n;
    uint64_t *d_kpow;
    Control *d_ctl;
    uint64_t *d_status;
    PendingLine *d_pending;
    uint32_t pending_cap;
};

extern "C" {

size_t sr_frame_datagram(uint8_t *dst, const uint8_t *src, size_t len) {
    // udp_read_cb: recv(fd, buffer, DATA_BUF_SIZE - 1, 0) (sr-main.c:163), then append '\n'
    // unless the datagram already ends with one (sr-main.c:171-173). Empty -> nothing (:170).
    size_t n = len < SR_MAX_DATAGRAM ? len : SR_MAX_DATAGRAM;
    if (n == 0) return 0;
    memcpy(dst, src, n);
    if (dst[n - 1] != '\n') dst[n++] = '\n';
    return n;
}

size_t sr_frame_datagrams(uint8_t *dst, size_t dst_cap, const uint8_t *const *dgrams,
                          const size_t *lens, size_t count) {
    size_t pos = 0;
    for (size_t i = 0; i < count; ++i) {
        const size_t need = (lens[i] < SR_MAX_DATAGRAM ? lens[i] : SR_MAX_DATAGRAM) + 1;
        if (pos + need > dst_cap) return (size_t)-1;
        pos += sr_frame_datagram(dst + pos, dgrams[i], lens[i]);
    }
    return pos;
}

const char *sr_version(void) {
    return "statsd-router-mi355x 0.1 (gfx950 route_kernel: 16 KiB tiles, decoupled look-back)";
}

static int upload_constants(int device) {
    if (device >= 0 && device < 64 && tables_uploaded[device]) return 0;
    uint64_t kp16[17], kinv[64], klane[64];
    for (int i = 0; i < 17; ++i) kp16[i] = ipow(K, (unsigned)i);
    uint64_t x = 1;
    for (int i = 0; i < 64; ++i) { kinv[i] = x; x *= kKinv; }
    for (int i = 0; i < 64; ++i) klane[i] = ipow(K, 64u * (unsigned)i);
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_kpow16), kp16, sizeof(kp16)) != hipSuccess) return -EIO;
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_kinv), kinv, sizeof(kinv)) != hipSuccess) return -EIO;
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_klane), klane, sizeof(klane)) != hipSuccess) return -EIO;
    if (device >= 0 && device < 64) tables_uploaded[device] = true;
    return 0;
}

void sr_close(sr_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(ctx->d_in);
    (void)hipFree(ctx->d_out);
    (void)hipFree(ctx->d_hash);
    (void)hipFree(ctx->d_count);
    (void)hipFree(ctx->d_alive);
    (void)hipFree(ctx->d_magic);
    (void)hipFree(ctx->d_kpow);
    (void)hipFree(ctx->d_ctl);
    (void)hipFree(ctx->d_status);
    (void)hipFree(ctx->d_pending);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    free(ctx->h_alive);
    free(ctx);
}

int sr_open(sr_ctx **out, int device, size_t max_batch_bytes, uint32_t n_downstreams) {
    if (!out) return -EINVAL;
    *out = nullptr;
    if (max_batch_bytes == 0 || max_batch_bytes > 0xFFFFFFF0ull || n_downstreams > SR_MAX_DOWNSTREAMS)
        return -EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return -ENODEV;
    if (hipSetDevice(device) != hipSuccess) return -ENODEV;
    sr_ctx *c = (sr_ctx *)calloc(1, sizeof(sr_ctx));
    if (!c) return -ENOMEM;
    c->device = device;
    c->max_batch = max_batch_bytes;
    c->nds = n_downstreams;
    c->nwords = (n_downstreams + 63) / 64;
    c->max_tiles = (uint32_t)((max_batch_bytes + kTile - 1) / kTile);
    c->h_alive = (uint64_t *)calloc(c->nwords ? c->nwords : 1, sizeof(uint64_t));
    int rc = -ENOMEM;
    if (!c->h_alive) goto fail;
    if (upload_constants(device) != 0) { rc = -EIO; goto fail; }
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) goto fail;
    c->stream = c->own_stream;
    if (hipMalloc(&c->d_in, max_batch_bytes) != hipSuccess) goto fail;
    if (hipMalloc(&c->d_count, sizeof(uint64_t)) != hipSuccess) goto fail;
    if (hipMalloc(&c->d_alive, (c->nwords ? c->nwords : 1) * sizeof(uint64_t)) != hipSuccess) goto fail;
    if (hipMalloc(&c->d_magic, (n_downstreams + 1) * sizeof(Magic)) != hipSuccess) goto fail;
    if (hipMalloc(&c->d_kpow, kPowTable * sizeof(uint64_t)) != hipSuccess) goto fail;
    if (hipMalloc(&c->d_ctl, sizeof(Control)) != hipSuccess) goto fail;
    if (hipMalloc(&c->d_status, c->max_tiles * sizeof(uint64_t)) != hipSuccess) goto fail;
    if (hipMemset(c->d_ctl, 0, sizeof(Control)) != hipSuccess) goto fail;
    if (hipMemset(c->d_status, 0, c->max_tiles * sizeof(uint64_t)) != hipSuccess) goto fail;
    {
        std::vector<Magic> mg(n_downstreams + 1);
        for (uint32_t d = 1; d <= n_downstreams; ++d) {
            mg[d] = make_magic(d);
            // self-check of the reciprocal against the hardware divide on awkward numerators
            const uint64_t probes[6] = {0ull, 1ull, d - 1ull, (uint64_t)d, ~0ull, 0x9E3779B97F4A7C15ull * d + 7};
            for (uint64_t nn : probes)
                if (host_div(nn, mg[d]) != nn / d) { rc = -EIO; goto fail; }
        }
        c->magic_n = n_downstreams ? mg[n_downstreams] : Magic{0, 0, 0};
        if (hipMemcpy(c->d_magic, mg.data(), mg.size() * sizeof(Magic), hipMemcpyHostToDevice) != hipSuccess)
            goto fail;
        std::vector<uint64_t> kp(kPowTable);
        uint64_t x = 1;
        for (int i = 0; i < kPowTable; ++i) { kp[i] = x; x *= K; }
        if (hipMemcpy(c->d_kpow, kp.data(), kp.size() * sizeof(uint64_t), hipMemcpyHostToDevice) != hipSuccess)
            goto fail;
    }
    for (uint32_t i = 0; i < n_downstreams; ++i) c->h_alive[i >> 6] |= 1ull << (i & 63);
    if (hipMemcpy(c->d_alive, c->h_alive, (c->nwords ? c->nwords : 1) * sizeof(uint64_t),
                  hipMemcpyHostToDevice) != hipSuccess)
        goto fail;
    c->dead = 0;
    *out = c;
    return 0;
fail:
    sr_close(c);
    return rc;
}

int sr_set_alive(sr_ctx *c, const uint64_t *alive) {
    if (!c || (!alive && c->nds)) return -EINVAL;
    (void)hipSetDevice(c->device);
    uint32_t live = 0;
    for (uint32_t w = 0; w < c->nwords; ++w) {
        uint64_t v = alive[w];
        if (w == c->nwords - 1 && (c->nds & 63)) v &= (1ull << (c->nds & 63)) - 1;
        c->h_alive[w] = v;
        live += (uint32_t)__builtin_popcountll(v);
    }
    c->dead = c->nds - live;
    if (c->nwords &&
        hipMemcpyAsync(c->d_alive, c->h_alive, c->nwords * sizeof(uint64_t), hipMemcpyHostToDevice,
                       c->stream) != hipSuccess)
        return -EIO;
    if (c->dead > (uint32_t)kOverlay && !c->d_pending) {
        c->pending_cap = (uint32_t)(c->max_batch / SR_MIN_LINE_LENGTH + 1);
        if (hipMalloc(&c->d_pending, (size_t)c->pending_cap * sizeof(PendingLine)) != hipSuccess) {
            c->d_pending = nullptr;
            c->pending_cap = 0;
            return -ENOMEM;
        }
    }
    // the copy reads h_alive: make it complete before the caller may touch the snapshot again
    return hipStreamSynchronize(c->stream) == hipSuccess ? 0 : -EIO;
}

int sr_set_stream(sr_ctx *c, void *stream) {
    if (!c) return -EINVAL;
    c->stream = stream ? (hipStream_t)stream : c->own_stream;
    return 0;
}

int sr_sync(sr_ctx *c) {
    if (!c) return -EINVAL;
    (void)hipSetDevice(c->device);
    return hipStreamSynchronize(c->stream) == hipSuccess ? 0 : -EIO;
}

int sr_route_device(sr_ctx *c, const uint8_t *d_bytes, size_t nbytes, sr_record *d_out,
                    size_t max_records, uint64_t *d_hashes, uint64_t *d_n_records) {
    if (!c || !d_n_records || (nbytes && !d_bytes) || nbytes > c->max_batch) return -EINVAL;
    if (max_records && !d_out) return -EINVAL;
    (void)hipSetDevice(c->device);
    if (nbytes == 0)
        return hipMemsetAsync(d_n_records, 0, sizeof(uint64_t), c->stream) == hipSuccess ? 0 : -EIO;
    RouteParams p;
    p.bytes = d_bytes;
    p.nbytes = (uint32_t)nbytes;
    p.ntiles = (uint32_t)((nbytes + kTile - 1) / kTile);
    p.recs = d_out;
    p.hashes = d_hashes;
    p.n_out = d_n_records;
    p.max_records = (uint32_t)(max_records > 0xFFFFFFFFull ? 0xFFFFFFFFull : max_records);
    p.nds = c->nds;
    p.dead = c->dead;
    p.pending_cap = c->pending_cap;
    p.magic_n = c->magic_n;
    p.alive = c->d_alive;
    p.magic = c->d_magic;
    p.kpow = c->d_kpow;
    p.ctl = c->d_ctl;
    p.status = c->d_status;
    p.pending = c->d_pending;
    const bool wide = c->dead > (uint32_t)kOverlay && c->dead < c->nds;
    if (wide && hipMemsetAsync(&c->d_ctl->pending, 0, sizeof(uint32_t), c->stream) != hipSuccess)
        return -EIO;
    hipLaunchKernelGGL(route_kernel, dim3(p.ntiles), dim3(kBlock), 0, c->stream, p);
    if (hipGetLastError() != hipSuccess) return -EIO;
    if (wide) {
        const size_t lds = (size_t)c->nds * sizeof(uint16_t);
        static bool attr_set = false;
        if (!attr_set) {
            (void)hipFuncSetAttribute((const void *)probe_wide_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
            attr_set = true;
        }
        hipLaunchKernelGGL(probe_wide_kernel, dim3(256), dim3(64), lds, c->stream, p);
        if (hipGetLastError() != hipSuccess) return -EIO;
    }
    return 0;
}

int sr_route_batch(sr_ctx *c, const uint8_t *bytes, size_t nbytes, sr_record *out,
                   size_t max_records, size_t *n_records, uint64_t *hashes) {
    if (!c || !n_records || (nbytes && !bytes) || nbytes > c->max_batch) return -EINVAL;
    if (max_records && !out) return -EINVAL;
    *n_records = 0;
    if (nbytes == 0) return 0;
    if (bytes[nbytes - 1] != '\n') return -EINVAL;
    (void)hipSetDevice(c->device);
    // device record capacity: never more lines than bytes
    const size_t cap = max_records < nbytes ? max_records : nbytes;
    if (cap > c->d_out_cap) {
        (void)hipFree(c->d_out);
        c->d_out = nullptr;
        c->d_out_cap = 0;
        if (hipMalloc(&c->d_out, cap * sizeof(sr_record)) != hipSuccess) return -ENOMEM;
        c->d_out_cap = cap;
    }
    if (hashes && cap > c->d_hash_cap) {
        (void)hipFree(c->d_hash);
        c->d_hash = nullptr;
        c->d_hash_cap = 0;
        if (hipMalloc(&c->d_hash, cap * sizeof(uint64_t)) != hipSuccess) return -ENOMEM;
        c->d_hash_cap = cap;
    }
    if (hipMemcpyAsync(c->d_in, bytes, nbytes, hipMemcpyHostToDevice, c->stream) != hipSuccess) return -EIO;
    int rc = sr_route_device(c, c->d_in, nbytes, c->d_out, cap, hashes ? c->d_hash : nullptr, c->d_count);
    if (rc) return rc;
    uint64_t n = 0;
    if (hipMemcpyAsync(&n, c->d_count, sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream) != hipSuccess)
        return -EIO;
    if (hipStreamSynchronize(c->stream) != hipSuccess) return -EIO;
    const size_t ncopy = n < cap ? (size_t)n : cap;
    if (ncopy) {
        if (hipMemcpyAsync(out, c->d_out, ncopy * sizeof(sr_record), hipMemcpyDeviceToHost, c->stream) !=
            hipSuccess)
            return -EIO;
        if (hashes && hipMemcpyAsync(hashes, c->d_hash, ncopy * sizeof(uint64_t), hipMemcpyDeviceToHost,
                                     c->stream) != hipSuccess)
            return -EIO;
        if (hipStreamSynchronize(c->stream) != hipSuccess) return -EIO;
    }
    *n_records = (size_t)n;
    return n > max_records ? -ENOSPC : 0;
}

}  // extern "C"
