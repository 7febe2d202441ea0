/*
 * sr_router.h — one data thread of the MI355X statsd-router, on top of the C ABI in sr_route.h.
 *
 * The reference runs one libev loop per data thread (data_pipe_thread, sr-main.c:237-308), each
 * with its own copy of the downstream array (sr-main.c:249): a 1450-byte active buffer per
 * downstream that lines are appended to (push_to_downstream, sr-main.c:73-83) and that is
 * flushed when the next line would not fit or on the flush timer (ds_schedule_flush /
 * ds_flush_timer_cb, sr-main.c:49-71,194-204), plus per-downstream traffic / packet counters and
 * the self-metrics of ping_cb (sr-main.c:206-235).
 *
 * sr_core is that per-thread state with the per-line work moved to the GPU: a batch of framed
 * datagrams is classified, hashed, shard-picked AND packed into per-downstream packets on the
 * device (sr_route_pack_batch); the host only walks the packet descriptors (one iovec per line),
 * drops the pending buffers of probed dead downstreams (sr-main.c:106) and formats the WARN
 * lines of invalid lines with the reference's exact texts (sr-main.c:115,142,184). Timers (flush,
 * ping) run on the host between batches, exactly as libev runs them between read callbacks.
 *
 * Conventions: 0 or a negative errno; not thread-safe (one sr_core per data thread).
 */
#ifndef SR_ROUTER_H
#define SR_ROUTER_H

#include <stddef.h>
#include <stdint.h>
#include <sys/uio.h>

#include "sr_route.h"

#ifdef __cplusplus
extern "C" {
#endif

/* log levels of the reference logger (sr-util.h:15-21) */
enum sr_log_level { SR_TRACE = 0, SR_DEBUG = 1, SR_INFO = 2, SR_WARN = 3, SR_ERROR = 4 };

#define SR_METRIC_SIZE 256u  /* sr-types.h:32: buffers of the ping metric names */

typedef struct sr_core_config {
    int device;                        /* HIP device of the thread's context                    */
    size_t max_batch_bytes;            /* framed bytes per sr_core_route call                    */
    uint32_t n_downstreams;            /* the `downstream=` list of statsd-router.conf           */
    const char *const *ds_hosts;       /* each downstream's host, as written in the config        */
    const char *const *ds_data_ports;  /* each downstream's data port, as written                 */
    const char *ping_prefix;           /* ping_prefix=                                             */
    const char *hostname;              /* gethostname() of the router (sr-init.c:298)             */
    int data_port;                     /* data_port + thread index: the names of sr-init.c:57,113 */
    int log_level;                     /* messages below this level are not even formatted        */
} sr_core_config;

/* A flushed packet for downstream ds: iov[0..iovcnt) concatenated, `bytes` in total (<= 1450).
 * The iovecs point into core-owned and caller-owned memory that later calls overwrite: the
 * callback must consume them (send or copy) before it returns. */
typedef void (*sr_core_emit_fn)(void *user, uint32_t ds, const struct iovec *iov, int iovcnt, size_t bytes);
/* A log message (no trailing newline, no timestamp: the text the reference passes to log_msg). */
typedef void (*sr_core_log_fn)(void *user, int level, const char *msg, size_t len);
/* Called once at the end of every call that may have emitted packets (e.g. to sendmmsg them). */
typedef void (*sr_core_flush_fn)(void *user);

typedef struct sr_core sr_core;
int sr_core_open(sr_core **core, const sr_core_config *cfg, sr_core_emit_fn emit, sr_core_log_fn log,
                 sr_core_flush_fn flush, void *user);

/* The health checker's alive bits (sr-types.h:25): ceil(n/64) words. All start DEAD, as in the
 * reference (sr-init.c:85). */
int sr_core_set_alive(sr_core *core, const uint64_t *alive);

/* A page-locked buffer of max_batch_bytes the caller may frame datagrams into (optional; it is slot
 * 0's buffer of the double-buffered calls below). */
uint8_t *sr_core_batch_buffer(sr_core *core, size_t *capacity);

/* Route one batch of framed datagrams (sr_frame_datagram output, back to back): what the
 * reference does in udp_read_cb for each datagram in turn (sr-main.c:149-191). */
int sr_core_route(sr_core *core, const uint8_t *framed, size_t nbytes);

/* Double-buffered routing: the host's work on one batch (walking its packets, the emit and log
 * callbacks, receiving the next datagrams) overlaps the GPU's work on the next (sr_route_pack_submit).
 * The core owns two page-locked batch buffers, slots 0 and 1 (sr_core_slot_buffer). sr_core_submit
 * starts routing slot `slot`'s first nbytes, then completes the OTHER slot's batch if one is in
 * flight (its packets are emitted, its WARN lines logged, the flush callback called), so when it
 * returns at most `slot` is in flight and the other slot's buffer may be refilled. sr_core_drain
 * completes the batch in flight, if any. Batches complete in submission order, with exactly the
 * packets, pending buffers, counters and log lines that sr_core_route would produce for them one
 * after another; pending bytes chain on the device between batches. sr_core_route,
 * sr_core_flush_timer, sr_core_ping and sr_core_set_alive drain first. Returns 0, -EBUSY (the slot is
 * in flight), -EINVAL or an sr_route_pack_* error. */
uint8_t *sr_core_slot_buffer(sr_core *core, int slot, size_t *capacity);
int sr_core_submit(sr_core *core, int slot, size_t nbytes);
int sr_core_drain(sr_core *core);

/* The same two calls with the batch's datagram boundaries: ends[i] is the end offset (exclusive) of
 * framed datagram i in the batch, ascending, the last = nbytes (empty datagrams have no entry: the
 * reference logs nothing for them, sr-main.c:170). Only a core opened at log_level SR_TRACE reads
 * them: it logs, in input order, "udp_read_cb: got packet ..." per datagram (sr-main.c:174) and, per
 * line that reaches find_downstream, its hash and first live pick (sr-main.c:91,102) between the WARN
 * lines, from the GPU's per-line hashes (sr_set_trace). Without boundaries (the calls above) a TRACE
 * core logs the per-line messages only. The array is copied; it may be reused on return. */
int sr_core_route_datagrams(sr_core *core, const uint8_t *framed, size_t nbytes, const uint32_t *ends,
                            size_t n_datagrams);
int sr_core_submit_datagrams(sr_core *core, int slot, size_t nbytes, const uint32_t *ends, size_t n_datagrams);

/* The core's device context (sr_route.h), e.g. for sr_set_layout or sr_set_knob (developer A/B runs).
 * Owned by the core. */
sr_ctx *sr_core_context(sr_core *core);

/* Test hook (fault injection; nothing calls it in the executable): the fail_submit-th call of
 * sr_core_submit* fails as a failed sr_route_pack_submit (the batch is not taken), and the
 * fail_finish-th batch to complete fails as a failed sr_route_pack_result (its packets and log lines
 * are lost; a batch submitted after it on device-chained fills is taken back and routed again from
 * the host's pending buffers). 0 = never. Counts start at this call. */
int sr_core_inject_faults(sr_core *core, unsigned fail_submit, unsigned fail_finish);

/* The slot whose batch is on the GPU (0 or 1), -1 if none, -EINVAL. After a failed sr_core_submit
 * it tells the caller whether the new batch was taken (the call can also fail after submitting it,
 * when completing the previous batch failed): a caller that refills the other slot only when
 * sr_core_in_flight() == slot never overwrites a batch still in flight. */
int sr_core_in_flight(const sr_core *core);

/* ds_flush_timer_cb (sr-main.c:194-204): flush every non-empty pending buffer. */
int sr_core_flush_timer(sr_core *core);

/* ping_cb (sr-main.c:206-235): per-downstream connection counters to live downstreams, traffic and
 * packet counters routed like data lines, then the healthy-downstreams gauge. */
int sr_core_ping(sr_core *core);

/* Pending (active) buffer and counters of downstream ds. */
int sr_core_state(const sr_core *core, uint32_t ds, const uint8_t **pending, size_t *len, int32_t *traffic,
                  int32_t *packets);

/* The ping metric names (sr-init.c:57,112-118): which = 0 per-downstream connections (two lines),
 * 1 traffic, 2 packets, 3 the thread's healthy-downstreams gauge (ds ignored). */
const char *sr_core_metric_name(const sr_core *core, uint32_t ds, int which);

void sr_core_close(sr_core *core);

#ifdef __cplusplus
}
#endif

#endif /* SR_ROUTER_H */
