/*
 * routing_filter_amd.h -- the calls the MI355X routing-filter shim adds to
 * src/routing_filter.h (shim/routing_filter_amd.c).
 */
#pragma once

#include "platform.h"
#include "routing_filter.h"

/* probe every routing_filter_lookup_async state queued so far in the caller's thread (one
 * GPU launch over every filter they name), complete them and fire their callbacks. Queued
 * states also complete on their own: the shim's completion thread takes the whole queue
 * whenever it is free (what arrived during its previous GPU round trip), waiting up to
 * RF_SHIM_ASYNC_WINDOW_US (default 0) microseconds for RF_SHIM_ASYNC_BATCH states */
void
routing_filter_amd_flush(void);

/* the completion thread's batch size and window (RF_SHIM_ASYNC_BATCH and
 * RF_SHIM_ASYNC_WINDOW_US at start-up) */
void
routing_filter_amd_async_config(uint64 batch, uint64 window_us);

/* flushes so far (GPU launches) and states completed */
void
routing_filter_amd_async_stats(uint64 *batches, uint64 *probes);

/* nanoseconds spent so far probing queued states (grouping, residency, the GPU round trip) */
uint64
routing_filter_amd_async_probe_ns(void);
/* out[0..5]: async batches, states, ns of the burst wait, batch gathering, lookup_many and
 * callbacks (diagnostics) */
void
routing_filter_amd_async_breakdown(uint64 *out);

/* routing_filter_add calls coalesced: GPU batches built and filters they held */
void
routing_filter_amd_add_stats(uint64 *batches, uint64 *filters);

/* device bytes held by the resident-filter registry (bound: RF_AMD_REGISTRY_MIB, default
 * 32768), filters evicted and batches trimmed to their probe-only state so far */
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
