/*
 * routing_filter_amd.h -- the two calls the MI355X routing-filter shim adds to
 * src/routing_filter.h (shim/routing_filter_amd.c).
 */
#pragma once

#include "platform.h"

/* probe every routing_filter_lookup_async state queued so far (one GPU probe per filter),
 * complete them and fire their callbacks; also happens on its own when RF_SHIM_ASYNC_BATCH
 * states are queued or a queued state is called again */
void
routing_filter_amd_flush(void);

/* flushes so far: GPU probe launches and states completed */
void
routing_filter_amd_async_stats(uint64 *batches, uint64 *probes);
