/*
 * TEST INFRASTRUCTURE ONLY (tests/test_ref_pinning.py). Compiles the reference's own
 * src/routing_filter.c -- #included from where it lies under /root/reference at build time
 * (oracle/Makefile), never copied -- so that its static helpers can be called directly:
 *   RadixSort                  src/routing_filter.c:54-131
 *   routing_get_bucket_bounds  src/routing_filter.c:230-279
 *   routing_get_bucket_counts  src/routing_filter.c:281-306
 * The pinning test fuzzes the restatement's equivalents (oracle/rf_oracle.c rfo_radix_sort,
 * rfo_bucket_bounds, rfo_bucket_counts) against these. Linked into _ref/libref_static.so
 * with the same page stack as _ref/libref_rf.so, in place of routing_filter.c.
 */
#include "routing_filter.c"

uint32 *
refs_radix_sort(uint32 *pData, uint32 *pTemp, uint32 count, uint32 fp_size)
{
   /* RadixSort asserts a zeroed histogram matrix (routing_filter.c:72-76) */
   uint32 mBuf[MATRIX_ROWS * MATRIX_COLS];
   memset(mBuf, 0, sizeof(mBuf));
   return RadixSort(pData, mBuf, pTemp, count, fp_size);
}

void
refs_bucket_bounds(char *encoding, uint64 len, uint64 bucket_offset, uint64 *start, uint64 *end)
{
   routing_get_bucket_bounds(encoding, len, bucket_offset, start, end);
}

void
refs_bucket_counts(uint32 log_index_size, routing_hdr *hdr, uint32 *count)
{
   routing_config cfg;
   memset(&cfg, 0, sizeof(cfg));
   cfg.log_index_size = log_index_size;
   cfg.index_size     = 1u << log_index_size;
   routing_get_bucket_counts(&cfg, hdr, count);
}
