/*
 * sr_gen.c — deterministic synthetic statsd traffic (host C, no GPU).
 *
 * The reference's own generator (statsd-traffic-generator.c:90-112) sends one ~19-byte
 * `test.counter<0..99>:1|c\n` datagram per timer tick and cannot produce the 64/256/1024-byte
 * metric shapes of the benchmark configs, so the build has its own. Line shapes follow the
 * reference's black-box tests (test/statsd-router-test-lib.rb:232-267):
 *   valid   : <name>:<value>|c\n
 *   invalid : (L-1) random [A-Z] + '\n'   (no ':' -> "invalid metric", or a bad length)
 * Lines are packed greedily, whole, into datagrams of at most max_dgram bytes (<= 4095, the
 * reference's recv cap, sr-main.c:163), so every datagram already ends in '\n' and framing is
 * the identity. The stream is the concatenation of the datagrams.
 *
 * PRNG: xorshift64* seeded by `seed` (seed = 0x5EED0000 + config number).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

enum { SR_GEN_FIXED = 0, SR_GEN_TEST_SHAPE = 1 };

typedef struct {
    uint64_t s;
} rng_t;

static inline uint64_t rng_next(rng_t *r) {
    uint64_t x = r->s;
    x ^= x >> 12;
    x ^= x << 25;
    x ^= x >> 27;
    r->s = x;
    return x * 0x2545F4914F6CDD1DULL;
}

static inline uint32_t rng_below(rng_t *r, uint32_t n) {
    return (uint32_t)(((rng_next(r) >> 32) * (uint64_t)n) >> 32);
}

static const char NAME_CHARS[] = "abcdefghijklmnopqrstuvwxyz0123456789._-";

/* Writes one line of exactly `len` bytes (len >= 6) into p. */
static void make_fixed_line(rng_t *r, uint8_t *p, uint32_t len, int invalid) {
    if (invalid) {
        for (uint32_t i = 0; i + 1 < len; i++) p[i] = (uint8_t)('A' + rng_below(r, 26));
        p[len - 1] = '\n';
        return;
    }
    uint32_t name_len = len - 5; /* ":1|c\n" */
    for (uint32_t i = 0; i < name_len; i++) p[i] = (uint8_t)NAME_CHARS[rng_below(r, 39)];
    memcpy(p + name_len, ":1|c\n", 5);
}

/* test/statsd-router-test-lib.rb:232-250 valid_metric(n): "statsd-cluster.count" + 'X' pad +
 * rand(100), exactly n name bytes, then ":<counter 0..999>|c". Returns the line length. */
static uint32_t make_test_shape_line(rng_t *r, uint8_t *p, uint32_t name_len, uint32_t *counter) {
    static const char base[] = "statsd-cluster.count";
    char num[4];
    uint32_t v = rng_below(r, 100);
    uint32_t nd = v >= 10 ? 2 : 1;
    num[0] = (char)('0' + (nd == 2 ? v / 10 : v));
    num[1] = (char)('0' + v % 10);
    uint32_t k = 0;
    memcpy(p, base, 20);
    k = 20;
    if (k + nd < name_len) {
        uint32_t pad = name_len - k - nd;
        memset(p + k, 'X', pad);
        k += pad;
    }
    memcpy(p + k, num, nd);
    k += nd;
    *counter = (*counter + 1) % 1000;
    char val[8];
    int vl = 0;
    uint32_t c = *counter;
    char tmp[4];
    int tl = 0;
    do {
        tmp[tl++] = (char)('0' + c % 10);
        c /= 10;
    } while (c);
    while (tl) val[vl++] = tmp[--tl];
    p[k++] = ':';
    memcpy(p + k, val, (size_t)vl);
    k += (uint32_t)vl;
    memcpy(p + k, "|c\n", 3);
    return k + 3;
}

/*
 * Fill `out` (capacity cap) with datagrams. kind SR_GEN_FIXED: each line's length is drawn
 * uniformly from lens[0..n_lens) and the line is invalid with probability p_invalid.
 * kind SR_GEN_TEST_SHAPE: lens[0] is the name length of valid_metric(n).
 * Stops before the first line that would overflow cap. Returns bytes written; the datagram
 * lengths go to dgram_lens (if not NULL, up to dgram_cap entries).
 */
size_t sr_gen_stream(uint64_t seed, uint32_t kind, const uint32_t *lens, uint32_t n_lens,
                     double p_invalid, uint32_t max_dgram, uint8_t *out, size_t cap,
                     uint32_t *dgram_lens, size_t dgram_cap, size_t *n_dgrams, size_t *n_lines) {
    rng_t r = {seed ? seed : 0x9E3779B97F4A7C15ULL};
    for (int i = 0; i < 4; i++) rng_next(&r);
    uint64_t thresh = (uint64_t)(p_invalid * 18446744073709551615.0);
    if (p_invalid <= 0.0) thresh = 0;
    size_t pos = 0, dstart = 0, nd = 0, nl = 0;
    uint32_t counter = 0;
    uint8_t line[8192];
    if (max_dgram == 0 || max_dgram > 65507) max_dgram = 4095;
    for (;;) {
        uint32_t len;
        if (kind == SR_GEN_TEST_SHAPE) {
            len = make_test_shape_line(&r, line, lens[0], &counter);
        } else {
            len = lens[n_lens > 1 ? rng_below(&r, n_lens) : 0];
            if (len < 6) len = 6;
            if (len > sizeof(line)) len = sizeof(line);
            int invalid = thresh && rng_next(&r) < thresh;
            make_fixed_line(&r, line, len, invalid);
        }
        if (pos + len > cap) break;
        if (pos - dstart + len > max_dgram && pos > dstart) { /* close the current datagram */
            if (dgram_lens && nd < dgram_cap) dgram_lens[nd] = (uint32_t)(pos - dstart);
            nd++;
            dstart = pos;
        }
        memcpy(out + pos, line, len);
        pos += len;
        nl++;
    }
    if (pos > dstart) {
        if (dgram_lens && nd < dgram_cap) dgram_lens[nd] = (uint32_t)(pos - dstart);
        nd++;
    }
    if (n_dgrams) *n_dgrams = nd;
    if (n_lines) *n_lines = nl;
    return pos;
}
