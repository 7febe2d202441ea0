/*
 * sr_host.h — internal declarations of the statsd-router-mi355x executable (host/): the
 * reference's host surface (config file, logger, downstream health checks, control port, data
 * threads with their timers) rebuilt in C around one sr_core (include/sr_router.h) per data thread.
 */
#ifndef SR_HOST_H
#define SR_HOST_H

#include <ev.h>
#include <netinet/in.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>

#include "../include/sr_router.h"

#define SR_HOST_NAME_SIZE 64                 /* sr-init.c:4 */
#define SR_LOG_BUF_SIZE 2048                 /* sr-util.h:13 */
#define SR_HEALTH_REQUEST "health"           /* sr-types.h:94 */
#define SR_HEALTH_RESPONSE_BUF_SIZE 32       /* sr-types.h:95 */
#define SR_HEALTH_UP_RESPONSE "health: up\n" /* sr-types.h:96 */
#define SR_HEALTH_CHECK_BUF_SIZE 32          /* sr-main.h:47 */
#define SR_CONTROL_REQUEST_BUF_SIZE 32       /* sr-main.h:48 */

/* ---- logger (sr-util.c:10-29) ---- */
extern int sr_log_level;
void sr_log(int level, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
void sr_log_text(int level, const char *msg, size_t len);

/* ---- downstream health (sr-health-client.c) ---- */
typedef struct sr_health_client {
    ev_io super;                 /* first: the watcher is the client (sr-types.h:17-26) */
    struct sockaddr_in sa_in;
    int id;
    int alive;
} sr_health_client;

/* ---- configuration (sr-init.c, sr-types.h:98-122) ---- */
typedef struct sr_config {
    int data_port, control_port;
    char *downstream_str;
    double downstream_health_check_interval, downstream_flush_interval, downstream_ping_interval;
    int threads_num, socket_out_num;
    char *ping_prefix;
    int downstream_num;
    char **ds_hosts, **ds_data_ports;           /* as written in the config */
    struct sockaddr_in *ds_addr;                /* data address of each downstream */
    sr_health_client *health_client;
    char hostname[SR_HOST_NAME_SIZE];
    char health_check_response_buf[SR_HEALTH_RESPONSE_BUF_SIZE];
    int health_check_response_buf_length;
    int control_socket;
    /* GPU side */
    size_t batch_bytes;                         /* framed bytes per sr_core_route call */
    int n_devices;
    int require_gpu;                            /* a data thread without a GPU ends the process */
    int dt_sync;                                /* SR_DT_SYNC=1: every read event routes and completes its */
                                                /* batch before returning (no double buffering; A/B)    */
    int dt_yield;                               /* full batches per read event before timers run (0: no cap) */
    double dt_yield_s;                          /* seconds per read event before timers run (0: no cap)  */
    /* alive bits published by the health checker to the data threads */
    _Atomic uint64_t alive_gen;
    _Atomic uint64_t *alive_words;
} sr_config;

int sr_init_config(const char *filename, sr_config *config);

/* ---- main-thread services ---- */
void sr_health_check_timer_cb(struct ev_loop *loop, ev_periodic *p, int revents);
typedef struct sr_health_timer {
    ev_periodic super;
    sr_config *config;
} sr_health_timer;

typedef struct sr_control_io {  /* ev_io_control, sr-types.h:9-15 */
    ev_io super;
    char *response;
    int response_len;
    char *health_response;
    int *health_response_len;
} sr_control_io;
void sr_control_accept_cb(struct ev_loop *loop, ev_io *watcher, int revents);

/* ---- data threads ---- */
void *sr_data_thread(void *arg);
typedef struct sr_thread {
    int index;
    pthread_t thread;
    sr_config *config;
} sr_thread;

#endif
