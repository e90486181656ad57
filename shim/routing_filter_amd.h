/*
 * routing_filter_amd.h -- the calls the MI355X routing-filter shim adds to
 * src/routing_filter.h (shim/routing_filter_amd.c).
 */
#pragma once

#include "platform.h"
#include "routing_filter.h"

/* probe every routing_filter_lookup_async state queued so far (one GPU round trip: a probe
 * per distinct filter), complete them and fire their callbacks; also happens on its own
 * when RF_SHIM_ASYNC_BATCH states are queued or a queued state is called again */
void
routing_filter_amd_flush(void);

/* flushes so far (GPU round trips) and states completed */
void
routing_filter_amd_async_stats(uint64 *batches, uint64 *probes);

/* n lookups (filters[i], keys[i]) in one GPU round trip -- the batch form of the per-bundle
 * routing_filter_lookup calls of trunk_merge_lookup (src/trunk.c:6008-6075): found[i] equals
 * what routing_filter_lookup(cc, cfg, &filters[i], keys[i], &found[i]) returns */
platform_status
routing_filter_amd_lookup_batch(cache                *cc,
                                const routing_config *cfg,
                                routing_filter       *filters,
                                const key            *keys,
                                uint64                n,
                                uint64               *found);
