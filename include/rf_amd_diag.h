/*
 * rf_amd_diag.h -- diagnostics of the MI355X routing-filter engine (librf_amd.so).
 *
 * Not part of the drop-in's product interface (include/rf_amd.h): hooks the parity tests and
 * the measurement tools use to look inside the engine. None of these has a counterpart in
 * the reference's src/routing_filter.h.
 */
#ifndef RF_AMD_DIAG_H
#define RF_AMD_DIAG_H

#include "rf_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* the batch's device-only probe lines (64 B each). read_lines copies them to host
 * (h_lines == NULL: only *num_lines is set); rebuild_lines re-cuts them from the filter
 * images with the image-upload kernel (k_plines), so a test can check that the build's
 * lines and the image's lines are byte-identical. */
int rf_amd_debug_read_lines(rf_amd_batch *b, uint8_t *h_lines, uint64_t bytes, uint64_t *num_lines);
int rf_amd_debug_rebuild_lines(rf_amd_batch *b);

/* the probe's memory floor, measured (bench.py `roofline.floor_ms`): one launch of a kernel
 * with k_probe's fast-path memory traffic and wave order over the same runs as
 * rf_amd_batch_probe_{keys,hashes}_runs (key_len 24: 16-byte-aligned keys; 4: hashes) --
 * key staging, one 64-B line gather per probe from its filter, one 8-byte store -- with the
 * hash and the decode replaced by a few integer operations. d_out receives no lookup results. */
int rf_amd_debug_probe_floor(rf_amd_batch *b, const void *d_in, uint32_t key_len, const uint64_t *h_counts,
                             uint64_t *d_out, void *stream);

/* diagnostics library only (librf_amd_stamps.so): a device buffer of 16 u64 per workgroup
 * (NULL = off); the instrumented kernel chosen by `kernel` (1 = bucket sort, 2 = fused
 * partition, 3 = page assembly, 4 = layout) stamps the shader clock at each of its phases
 * into it (tools/phase_times.py). The product library accepts only NULL. */
int rf_amd_debug_phase_buffer(void *d_buf, uint32_t kernel);

/* where the host-buffer lookup round trips (rf_amd_probe_filters_host and the forms built on
 * it) spent their time so far: out[0] calls, out[1] ns before the launch (lookup slot,
 * buffers, ordering after builds, argument packing), out[2] ns in the launch call, out[3] ns
 * waiting for the kernel's completion word and copying the results out. reset != 0 zeroes
 * the counters after reading them. */
int rf_amd_diag_lookup_stats(uint64_t *out, int reset);

/* the lookup server so far: out[0] tickets issued, out[1] server launches, out[2] the first
 * ticket the last exited server did not serve */
int rf_amd_lookup_server_stats(rf_amd_engine *e, uint64_t *out);

/* where the engine's lookup server keeps its request ring: 1 device memory written through the
 * BAR, 0 pinned host memory (RF_AMD_SRV_RING=host, or a box whose BAR mapping failed the
 * check), -1 no server yet */
int rf_amd_diag_lookup_ring(rf_amd_engine *e);

/* stops the engine's lookup server (its wave exits; relaunched waves exit at once) and, gap_us
 * microseconds later, marks it dead with error `err`, exactly as a failed launch or a faulted
 * server stream does: tickets published in the gap are never answered (tests of the error
 * path: every submitted tag must come back through rf_amd_lookup_reap or
 * rf_amd_lookup_server_failed) */
int rf_amd_diag_lookup_server_kill(rf_amd_engine *e, int err, uint32_t gap_us);

/* the source id the library was built from (16 hex digits of SHA-256 over the engine's
 * sources and headers, splinterdb_amd/build.py source_id): the Python loader refuses a
 * library whose id differs from the tree's (a stale prebuilt .so) */
const char *rf_amd_build_id(void);

#ifdef __cplusplus
}
#endif
#endif
