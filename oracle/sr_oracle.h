/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see sr_oracle.c). CPU restatement of the reference hot
 * path; the record layout is the one of include/sr_route.h so outputs compare byte for byte.
 */
#ifndef SR_ORACLE_H
#define SR_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/sr_route.h"

size_t sro_frame_datagram(uint8_t *dst, const uint8_t *src, size_t len);
int sro_hash(const uint8_t *s, size_t length, uint64_t *out);
int sro_find_downstream(uint64_t hash, uint32_t downstream_num, const uint64_t *alive);
size_t sro_route_batch(const uint8_t *buf, size_t nbytes, uint32_t downstream_num,
                       const uint64_t *alive, sr_record *out, size_t max_records,
                       uint64_t *hashes);
size_t sro_route_datagrams(const uint8_t *dgrams, const uint32_t *lens, size_t count,
                           uint8_t *framed, size_t framed_cap, size_t *framed_len,
                           uint32_t downstream_num, const uint64_t *alive, sr_record *out,
                           size_t max_records, uint64_t *hashes);
void sro_probed_dead(const uint8_t *buf, size_t nbytes, uint32_t downstream_num,
                     const uint64_t *alive, uint64_t *probed);
int sro_pack_packets(const sr_record *recs, size_t n, uint32_t nds, const uint16_t *fill_in,
                     const uint64_t *probed_dead, sr_record *sorted, sr_packet *packets,
                     size_t max_packets, size_t *n_packets, size_t *n_valid, uint16_t *fill_out);
int sro_bench(const uint8_t *const *batches, const size_t *sizes, size_t nbatch, uint32_t nds,
              const uint64_t *alive, int threads, double seconds, uint64_t *lines,
              uint64_t *bytes, double *wall);

#endif
