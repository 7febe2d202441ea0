/*
 * sr_config.c — statsd-router.conf and the logger, with the reference's rules and messages so
 * that existing config files, init scripts and log watchers keep working:
 *   log_msg            sr-util.c:10-29    "YYYY-mm-dd HH:MM:SS <tid> <LEVEL> <message>" on stdout
 *   init_config        sr-init.c:241-331  key=value lines, '#' comments, defaults, verification
 *   process_config_line sr-init.c:126-174
 *   verify_config      sr-init.c:187-222
 *   init_downstream    sr-init.c:21-123   host:data_port:health_port,... (list order = shard id)
 */
#define _GNU_SOURCE
#include <errno.h>
#include <netdb.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/resource.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include "sr_host.h"

int sr_log_level = SR_TRACE;

static const char *level_name(int level) {
    static const char *names[] = {"TRACE", "DEBUG", "INFO", "WARN", "ERROR"};
    return level >= 0 && level <= SR_ERROR ? names[level] : "?";
}

/* timestamp, thread id and level prefix; returns its length (sr-util.c:20-24) */
static int log_prefix(char *buf, int level) {
    time_t t;
    struct tm tm;
    time(&t);
    localtime_r(&t, &tm);
    int l = (int)strftime(buf, SR_LOG_BUF_SIZE, "%Y-%m-%d %H:%M:%S", &tm);
    l += snprintf(buf + l, SR_LOG_BUF_SIZE - l, " %ld %s ", (long)syscall(SYS_gettid), level_name(level));
    return l;
}

void sr_log(int level, const char *fmt, ...) {
    if (level < sr_log_level) return;
    char buf[SR_LOG_BUF_SIZE];
    const int l = log_prefix(buf, level);
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf + l, SR_LOG_BUF_SIZE - l, fmt, ap);
    va_end(ap);
    fprintf(stdout, "%s\n", buf);
    fflush(stdout);
}

/* a message formatted elsewhere (the data threads' WARN lines), truncated like vsnprintf would */
void sr_log_text(int level, const char *msg, size_t len) {
    if (level < sr_log_level) return;
    char buf[SR_LOG_BUF_SIZE];
    const int l = log_prefix(buf, level);
    size_t room = SR_LOG_BUF_SIZE - (size_t)l - 1;
    size_t n = strnlen(msg, len < room ? len : room);
    memcpy(buf + l, msg, n);
    buf[l + n] = 0;
    fprintf(stdout, "%s\n", buf);
    fflush(stdout);
}

static char *dup_value(const char *v) {
    size_t n = strlen(v) + 1;
    char *p = malloc(n);
    if (p) memcpy(p, v, n);
    return p;
}

/* process_config_line: one "key=value" line; 0 ok, 1 failure (already logged) */
static int config_line(char *line, sr_config *c) {
    char *value = strchr(line, '=');
    if (!value) {
        sr_log(SR_ERROR, "%s: bad line in config \"%s\"", "process_config_line", line);
        return 1;
    }
    *value++ = 0;
    if (!strcmp(line, "data_port")) {
        c->data_port = atoi(value);
    } else if (!strcmp(line, "control_port")) {
        c->control_port = atoi(value);
    } else if (!strcmp(line, "downstream_flush_interval")) {
        c->downstream_flush_interval = atof(value);
    } else if (!strcmp(line, "downstream_health_check_interval")) {
        c->downstream_health_check_interval = atof(value);
    } else if (!strcmp(line, "downstream_ping_interval")) {
        c->downstream_ping_interval = atof(value);
    } else if (!strcmp(line, "log_level")) {
        sr_log_level = atoi(value);
    } else if (!strcmp(line, "threads_num")) {
        c->threads_num = atoi(value);
        if (c->threads_num < 1) {
            sr_log(SR_ERROR, "%s: threads_num should be >= 1", "process_config_line");
            return 1;
        }
    } else if (!strcmp(line, "ping_prefix")) {
        free(c->ping_prefix);
        if (!(c->ping_prefix = dup_value(value))) {
            sr_log(SR_ERROR, "%s: malloc() failed", "process_config_line");
            return 1;
        }
    } else if (!strcmp(line, "downstream")) {
        free(c->downstream_str);
        if (!(c->downstream_str = dup_value(value))) {
            sr_log(SR_ERROR, "%s: malloc() failed", "process_config_line");
            return 1;
        }
    } else {
        sr_log(SR_ERROR, "%s: unknown parameter \"%s\"", "process_config_line", line);
        return 1;
    }
    return 0;
}

static int verify(const sr_config *c) {
    int f = 0;
    const char *fn = "verify_config";
    if (c->data_port == 0) f++, sr_log(SR_ERROR, "%s: data_port not set", fn);
    if (c->control_port == 0) f++, sr_log(SR_ERROR, "%s: control_port not set", fn);
    if (sr_log_level < SR_TRACE || sr_log_level > SR_ERROR)
        f++, sr_log(SR_ERROR, "%s: log_level should be in the %d-%d range", fn, SR_TRACE, SR_ERROR);
    if (!c->downstream_str) f++, sr_log(SR_ERROR, "%s: downstream is not set", fn);
    if (!c->ping_prefix) f++, sr_log(SR_ERROR, "%s: ping_prefix is not set", fn);
    if (c->downstream_health_check_interval <= 0.0)
        f++, sr_log(SR_ERROR, "%s: downstream_health_check_interval should be > 0", fn);
    if (c->downstream_flush_interval <= 0.0) f++, sr_log(SR_ERROR, "%s: downstream_flush_interval should be > 0", fn);
    if (c->downstream_ping_interval <= 0.0) f++, sr_log(SR_ERROR, "%s: downstream_ping_interval should be > 0", fn);
    return f;
}

static int resolve(struct sockaddr_in *sa, const char *host, const char *port) {
    struct addrinfo hints, *res = NULL;
    memset(&hints, 0, sizeof(hints));
    hints.ai_family = AF_INET;
    if (getaddrinfo(host, NULL, &hints, &res) != 0 || !res) {
        sr_log(SR_ERROR, "%s: gethostbyname() failed %s", "init_sockaddr_in", strerror(errno));
        return 1;
    }
    memset(sa, 0, sizeof(*sa));
    sa->sin_family = AF_INET;
    sa->sin_port = htons((uint16_t)atoi(port));
    sa->sin_addr = ((struct sockaddr_in *)res->ai_addr)->sin_addr;
    freeaddrinfo(res);
    return 0;
}

/* init_downstream: the downstream list; its order is the shard numbering */
static int downstreams(sr_config *c) {
    const char *fn = "init_downstream";
    int n = 1;
    for (const char *p = c->downstream_str; *p; p++) n += *p == ',';
    c->downstream_num = n;
    c->ds_hosts = calloc((size_t)n, sizeof(char *));
    c->ds_data_ports = calloc((size_t)n, sizeof(char *));
    c->ds_addr = calloc((size_t)n, sizeof(struct sockaddr_in));
    c->health_client = calloc((size_t)n, sizeof(sr_health_client));
    c->alive_words = calloc((size_t)(n + 63) / 64, sizeof(uint64_t));
    if (!c->ds_hosts || !c->ds_data_ports || !c->ds_addr || !c->health_client || !c->alive_words) {
        sr_log(SR_ERROR, "%s: downstream malloc() failed %s", fn, strerror(errno));
        return 1;
    }
    char *host = c->downstream_str;
    for (int i = 0; i < n; i++) {
        if (!host) {
            sr_log(SR_ERROR, "%s: null hostname at iteration %d", fn, i);
            return 1;
        }
        char *next = strchr(host, ',');
        if (next) *next++ = 0;
        char *data_port = strchr(host, ':');
        if (!data_port) {
            sr_log(SR_ERROR, "%s: no data port for %s", fn, host);
            return 1;
        }
        *data_port++ = 0;
        char *health_port = strchr(data_port, ':');
        if (!health_port) {
            sr_log(SR_ERROR, "%s: no health_port for %s", fn, host);
            return 1;
        }
        *health_port++ = 0;
        sr_health_client *hc = &c->health_client[i];
        hc->super.fd = -1;
        hc->id = i;
        hc->alive = 0;
        if (resolve(&hc->sa_in, host, health_port) || resolve(&c->ds_addr[i], host, data_port)) return 1;
        c->ds_hosts[i] = host;
        c->ds_data_ports[i] = data_port;
        host = next;
    }
    return 0;
}

int sr_init_config(const char *filename, sr_config *c) {
    memset(c, 0, sizeof(*c));
    sr_log_level = SR_TRACE;
    c->threads_num = 1;
    c->control_socket = -1;
    FILE *f = fopen(filename, "rt");
    if (!f) {
        sr_log(SR_ERROR, "%s: fopen() failed %s", "init_config", strerror(errno));
        return 1;
    }
    char *line = NULL;
    size_t cap = 0;
    ssize_t l;
    int failures = 0;
    while ((l = getline(&line, &cap, f)) > 0) {
        if (line[l - 1] == '\n') line[l - 1] = 0;
        /* sr-init.c:271 tests buffer[0] != '\n' after that '\n' became NUL: an empty line is
         * therefore parsed, and rejected as a bad line; only '#' lines are skipped */
        if (line[0] != '#') failures += config_line(line, c);
    }
    free(line);
    fclose(f);
    if (failures > 0) {
        sr_log(SR_ERROR, "%s: failed to load config file", "init_config");
        return 1;
    }
    if (verify(c) != 0) {
        sr_log(SR_ERROR, "%s: failed to verify config file", "init_config");
        return 1;
    }
    if (gethostname(c->hostname, SR_HOST_NAME_SIZE) < 0) {
        sr_log(SR_ERROR, "%s: gethostname() failed", "init_config");
        return 1;
    }
    c->hostname[SR_HOST_NAME_SIZE - 1] = 0;
    if (downstreams(c) != 0) {
        sr_log(SR_ERROR, "%s: init_downstream() failed", "init_config");
        return 1;
    }
    /* outgoing sockets per thread from the descriptor limit (sr-init.c:307-327) */
    struct rlimit rl;
    if (getrlimit(RLIMIT_NOFILE, &rl) != 0) {
        sr_log(SR_ERROR, "%s: getrlimit() failed", "init_config");
        return 1;
    }
    const long free_fds = ((long)rl.rlim_cur - 3 - 1 - c->downstream_num - c->threads_num) / c->threads_num;
    if (free_fds < 1) {
        sr_log(SR_ERROR, "%s: socket_out_num should be >= 1", "init_config");
        return 1;
    }
    if (free_fds > c->downstream_num) {
        c->socket_out_num = c->downstream_num;
    } else {
        c->socket_out_num = (int)free_fds;
        sr_log(SR_WARN,
               "%s: %d downstreams are present but only %d free file handles, some downstreams will share outgoing "
               "sockets",
               "init_config", c->downstream_num, c->socket_out_num);
    }
    memcpy(c->health_check_response_buf, SR_HEALTH_UP_RESPONSE, sizeof(SR_HEALTH_UP_RESPONSE) - 1);
    c->health_check_response_buf_length = (int)sizeof(SR_HEALTH_UP_RESPONSE) - 1;
    return 0;
}
