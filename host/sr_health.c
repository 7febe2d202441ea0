/*
 * sr_health.c — the main thread's services, with the reference's protocol and messages:
 *   downstream health checks  sr-health-client.c:1-116  periodic non-blocking TCP connect, send
 *                             "health", expect the prefix "health: up\n"; the alive bits feed
 *                             every data thread's GPU context (published with a generation count)
 *   control port              sr-control-server.c:1-104  "health" -> the current reply;
 *                             "health <status>" -> sets the reply to "health: <status>\n" (LB drain)
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <unistd.h>

#include "sr_host.h"

static sr_config *g_config;   /* the process's configuration (one per process, like the reference's) */

static void publish_alive(sr_config *c) {
    const int n = c->downstream_num;
    for (int w = 0; w < (n + 63) / 64; w++) {
        uint64_t v = 0;
        for (int k = w * 64; k < n && k < w * 64 + 64; k++) v |= (uint64_t)(c->health_client[k].alive & 1) << (k & 63);
        atomic_store_explicit(&c->alive_words[w], v, memory_order_relaxed);
    }
    atomic_fetch_add_explicit(&c->alive_gen, 1, memory_order_release);
}

static int set_nonblock(int fd) { return fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK); }

static void mark_down(ev_io *w) {   /* ds_mark_down, sr-health-client.c:9-19 */
    sr_health_client *hc = (sr_health_client *)w;
    if (w->fd > 0) {
        close(w->fd);
        w->fd = -1;
    }
    if (hc->alive == 1) {
        hc->alive = 0;
        sr_log(SR_DEBUG, "%s downstream %d is down", "ds_mark_down", hc->id);
        publish_alive(g_config);
    }
}

static void health_read_cb(struct ev_loop *loop, ev_io *w, int revents) {   /* :21-41 */
    (void)revents;
    sr_health_client *hc = (sr_health_client *)w;
    char buf[SR_HEALTH_CHECK_BUF_SIZE + 1];
    ev_io_stop(loop, w);
    ssize_t n = recv(w->fd, buf, SR_HEALTH_CHECK_BUF_SIZE, 0);
    if (n <= 0) {
        sr_log(SR_WARN, "%s: recv() failed %s", "ds_health_read_cb", strerror(errno));
        mark_down(w);
        return;
    }
    buf[n] = 0;
    if (memcmp(buf, SR_HEALTH_UP_RESPONSE, sizeof(SR_HEALTH_UP_RESPONSE) - 1) != 0) {
        mark_down(w);
        return;
    }
    if (hc->alive == 0) {
        hc->alive = 1;
        sr_log(SR_DEBUG, "%s downstream %d is up", "ds_health_read_cb", hc->id);
        publish_alive(g_config);
    }
}

static void health_send_cb(struct ev_loop *loop, ev_io *w, int revents) {   /* :43-54 */
    (void)revents;
    const int fd = w->fd;
    ev_io_stop(loop, w);
    if (send(fd, SR_HEALTH_REQUEST, sizeof(SR_HEALTH_REQUEST) - 1, MSG_NOSIGNAL) <= 0) {
        sr_log(SR_WARN, "%s: send() failed %s", "ds_health_send_cb", strerror(errno));
        mark_down(w);
        return;
    }
    ev_io_init(w, health_read_cb, fd, EV_READ);
    ev_io_start(loop, w);
}

static void health_connect_cb(struct ev_loop *loop, ev_io *w, int revents) {   /* :56-70 */
    (void)revents;
    int err = 0;
    socklen_t len = sizeof(err);
    ev_io_stop(loop, w);
    getsockopt(w->fd, SOL_SOCKET, SO_ERROR, &err, &len);
    if (err) {
        mark_down(w);
        return;
    }
    ev_io_init(w, health_send_cb, w->fd, EV_WRITE);
    ev_io_start(loop, w);
}

void sr_health_check_timer_cb(struct ev_loop *loop, ev_periodic *p, int revents) {   /* :74-116 */
    (void)revents;
    sr_config *c = ((sr_health_timer *)p)->config;
    g_config = c;
    for (int i = 0; i < c->downstream_num; i++) {
        ev_io *w = &c->health_client[i].super;
        int fd = w->fd;
        if (fd > 0 && ev_is_active(w)) {
            sr_log(SR_WARN, "%s: previous health check request was not completed for downstream %d",
                   "ds_health_check_timer_cb", i);
            ev_io_stop(loop, w);
            mark_down(w);
            fd = -1;
        }
        if (fd < 0) {
            if ((fd = socket(AF_INET, SOCK_STREAM, 0)) == -1) {
                sr_log(SR_WARN, "%s: socket() failed %s", "ds_health_check_timer_cb", strerror(errno));
                continue;
            }
            if (set_nonblock(fd) == -1) {
                close(fd);
                sr_log(SR_WARN, "%s: setnonblock() failed %s", "ds_health_check_timer_cb", strerror(errno));
                continue;
            }
            if (connect(fd, (struct sockaddr *)&c->health_client[i].sa_in, sizeof(struct sockaddr_in)) == -1 &&
                errno == EINPROGRESS) {
                ev_io_init(w, health_connect_cb, fd, EV_WRITE);
            } else {
                sr_log(SR_WARN, "%s: connect() failed %s", "ds_health_check_timer_cb", strerror(errno));
                close(fd);
                continue;
            }
        } else {
            ev_io_init(w, health_send_cb, fd, EV_WRITE);
        }
        ev_io_start(loop, w);
    }
}

/* ---- control port ------------------------------------------------------------------------ */
static void control_read_cb(struct ev_loop *loop, ev_io *w, int revents);

static void control_write_cb(struct ev_loop *loop, ev_io *w, int revents) {   /* sr-control-server.c:5-30 */
    sr_control_io *cw = (sr_control_io *)w;
    if (EV_ERROR & revents) {
        sr_log(SR_WARN, "%s: invalid event %s", "control_write_cb", strerror(errno));
        return;
    }
    ev_io_stop(loop, w);
    if (cw->response_len > 0) {
        if (send(w->fd, cw->response, (size_t)cw->response_len, MSG_NOSIGNAL) > 0) {
            ev_io_init(w, control_read_cb, w->fd, EV_READ);
            ev_io_start(loop, w);
            return;
        }
        sr_log(SR_WARN, "%s: error while sending control response", "control_write_cb");
    } else {
        sr_log(SR_WARN, "%s: nothing to send", "control_write_cb");
    }
    close(w->fd);
    free(cw);
}

static void control_read_cb(struct ev_loop *loop, ev_io *w, int revents) {   /* :32-75 */
    sr_control_io *cw = (sr_control_io *)w;
    char req[SR_CONTROL_REQUEST_BUF_SIZE];
    if (EV_ERROR & revents) {
        sr_log(SR_WARN, "%s: invalid event %s", "control_read_cb", strerror(errno));
        return;
    }
    ev_io_stop(loop, w);
    ssize_t n = recv(w->fd, req, SR_CONTROL_REQUEST_BUF_SIZE - 1, 0);
    if (n > 0) {
        while (n > 0 && (req[n - 1] == '\n' || req[n - 1] == ' ')) n--;
        req[n] = 0;
        const char *space = memchr(req, ' ', (size_t)n);
        const ssize_t cmd = space ? space - req : n;
        cw->response_len = 0;
        if (cmd == (ssize_t)sizeof(SR_HEALTH_REQUEST) - 1 && !strncmp(req, SR_HEALTH_REQUEST, (size_t)cmd)) {
            /* "health <status>": the new (sticky) reply keeps the space: "health: <status>\n" */
            if (space)
                *cw->health_response_len =
                    snprintf(cw->health_response, SR_HEALTH_RESPONSE_BUF_SIZE, "%s:%s\n", SR_HEALTH_REQUEST, space);
            if (*cw->health_response_len >= SR_HEALTH_RESPONSE_BUF_SIZE)
                *cw->health_response_len = SR_HEALTH_RESPONSE_BUF_SIZE - 1;
            cw->response = cw->health_response;
            cw->response_len = *cw->health_response_len;
        }
        ev_io_init(w, control_write_cb, w->fd, EV_WRITE);
        ev_io_start(loop, w);
        return;
    }
    sr_log(SR_WARN, "%s: error while reading health check request", "control_read_cb");
    close(w->fd);
    free(cw);
}

void sr_control_accept_cb(struct ev_loop *loop, ev_io *w, int revents) {   /* :77-104 */
    if (EV_ERROR & revents) {
        sr_log(SR_WARN, "%s: invalid event %s", "control_accept_cb", strerror(errno));
        return;
    }
    sr_control_io *lw = (sr_control_io *)w;
    sr_control_io *cw = malloc(sizeof(*cw));
    if (!cw) {
        sr_log(SR_ERROR, "%s: malloc() failed %s", "control_accept_cb", strerror(errno));
        return;
    }
    cw->health_response = lw->health_response;
    cw->health_response_len = lw->health_response_len;
    struct sockaddr_in a;
    socklen_t al = sizeof(a);
    const int fd = accept(w->fd, (struct sockaddr *)&a, &al);
    if (fd < 0) {
        sr_log(SR_ERROR, "%s: accept() failed %s", "control_accept_cb", strerror(errno));
        free(cw);
        return;
    }
    ev_io_init(&cw->super, control_read_cb, fd, EV_READ);
    ev_io_start(loop, &cw->super);
}
