/*
 * routing_filter_amd.h -- the calls the MI355X routing-filter shim adds to
 * src/routing_filter.h (shim/routing_filter_amd.c).
 */
#pragma once

#include "platform.h"
#include "routing_filter.h"

/* complete every routing_filter_lookup_async state submitted so far in the caller's thread
 * (answers reaped from the engine's lookup server, batched states probed; callbacks fired).
 * States also complete on their own: the shim's completion threads reap answers and answer
 * batches as they arrive */
void
routing_filter_amd_flush(void);

/* reaps that completed states so far, and states completed */
void
routing_filter_amd_async_stats(uint64 *batches, uint64 *probes);

/* nanoseconds spent so far reaping answered states */
uint64
routing_filter_amd_async_probe_ns(void);
/* out[0..5]: reaps, states, ns submitting (hash, pin, ring), -, reaping, callbacks
 * (diagnostics) */
void
routing_filter_amd_async_breakdown(uint64 *out);

/* out[0..10]: routing_filter_add calls, combiner batches, then ns totals: batch creation,
 * staging copies, build, info read-back, image read-back (per batch); the wait for the batch,
 * page allocation and fill (per add); the one-time costs: engine creation, cache-buffer
 * registrations -- diagnostics */
void
routing_filter_amd_add_breakdown(uint64 *out);

/* routing_filter_add calls coalesced: GPU batches built and filters they held */
void
routing_filter_amd_add_stats(uint64 *batches, uint64 *filters);

/* device bytes held by the resident-filter registry (bound: RF_AMD_REGISTRY_MIB, default
 * 8192), filters evicted and batches trimmed to their probe-only state so far */
void
routing_filter_amd_registry_stats(uint64 *bytes, uint64 *evictions, uint64 *trims);

/* sets the registry's bound (MiB; RF_AMD_REGISTRY_MIB at start-up) and applies it now */
void
routing_filter_amd_registry_set_limit(uint64 mib);

/* n lookups (filters[i], keys[i]) in one GPU launch -- the batch form of the per-bundle
 * routing_filter_lookup calls of trunk_merge_lookup (src/trunk.c:6008-6075): found[i] equals
 * what routing_filter_lookup(cc, cfg, &filters[i], keys[i], &found[i]) returns */
platform_status
routing_filter_amd_lookup_batch(cache                *cc,
                                const routing_config *cfg,
                                routing_filter       *filters,
                                const key            *keys,
                                uint64                n,
                                uint64               *found);

/* Direct placement (optional). By default routing_filter_add reads each image back into a
 * pinned bounce buffer and copies it into the cache pages it allocated. After
 * routing_filter_amd_cache_attach(cc) -- called once the store is open; it also creates the
 * engine -- cc's page buffer is registered with the GPU and images are written straight into
 * its pages (RF_SHIM_DIRECT=0 keeps the bounce path). A caller that attaches a cache must call
 * routing_filter_amd_cache_release(cc) before the cache's buffer is unmapped
 * (splinterdb_close): release waits for the adds placing through it, then unregisters. The
 * unmodified reference calls neither and gets the bounce path: a registration is never made
 * behind the caller's back, because a GPU store into a buffer unmapped under its registration
 * is a GPU memory fault. attach returns 0 when the cache is attached, -1 when the bounce path
 * stays (no GPU, a buffer over RF_SHIM_DIRECT_MAX_MIB, or the registration failed). */
int
routing_filter_amd_cache_attach(cache *cc);

void
routing_filter_amd_cache_release(cache *cc);

/* out[0]: caches registered now; out[1]: registrations a placement found stale; out[2]: adds
 * placing through a registration now */
void
routing_filter_amd_direct_stats(uint64 *out);
