/*
 * abi_smoke.c -- a plain C client of librf_amd.so through include/rf_amd.h (no ctypes, no
 * Python): the link-level check of the C ABI. Built by __graft_entry__.build() into
 * tests/c/abi_smoke. Without a HIP device it checks the host helpers and that engine
 * creation fails with ENODEV (no CPU fallback); with one (--expect-gpu) it builds a filter
 * from host hashes with rf_amd_filter_add (routing_filter_add's replacement), looks every
 * hash up, and checks the false-positive rate of never-inserted hashes.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "rf_amd.h"

static uint32_t
xorshift(uint64_t *s)
{
   *s ^= *s << 13;
   *s ^= *s >> 7;
   *s ^= *s << 17;
   return (uint32_t)(*s >> 32);
}

int
main(int argc, char **argv)
{
   const int     expect_gpu = argc > 1 && strcmp(argv[1], "--expect-gpu") == 0;
   rf_amd_config cfg        = {26, 8, 42, 4096, 32};
   if (rf_amd_max_fingerprints(&cfg) != 8388607ull) {
      fprintf(stderr, "max_fingerprints %llu\n", (unsigned long long)rf_amd_max_fingerprints(&cfg));
      return 1;
   }
   if (rf_amd_estimate_unique_keys_from_count(&cfg, 992680) != 1000095u) {
      fprintf(stderr, "estimate_unique_keys_from_count\n");
      return 1;
   }
   rf_amd_engine *e  = NULL;
   int            rc = rf_amd_engine_create(0, &e);
   if (rc == RF_AMD_ENODEV) {
      printf("abi_smoke: host helpers OK; no HIP device: ENODEV (%s)\n", rf_amd_last_error());
      return expect_gpu ? 1 : 0;
   }
   if (rc) {
      fprintf(stderr, "engine: %d %s\n", rc, rf_amd_last_error());
      return 1;
   }
   const uint64_t n  = 100000;
   uint32_t      *h  = malloc(4 * 2 * n);
   uint64_t      *fv = malloc(8 * 2 * n);
   uint64_t       st = 0x9E3779B97F4A7C15ull;
   for (uint64_t i = 0; i < 2 * n; i++) {
      h[i] = xorshift(&st);
   }
   rf_amd_image f;
   rc = rf_amd_filter_add(e, &cfg, NULL, &f, h, n, 5);
   if (rc) {
      fprintf(stderr, "filter_add: %d %s\n", rc, rf_amd_last_error());
      return 1;
   }
   rc = rf_amd_filter_lookup_hashes(e, &cfg, &f, h, 2 * n, fv);
   if (rc) {
      fprintf(stderr, "lookup: %d %s\n", rc, rf_amd_last_error());
      return 1;
   }
   uint64_t missing = 0, fp = 0;
   for (uint64_t i = 0; i < n; i++) {
      missing += !((fv[i] >> 5) & 1);
   }
   for (uint64_t i = n; i < 2 * n; i++) {
      fp += fv[i] != 0;
   }
   printf("abi_smoke: filter of %u fingerprints, %u unique, %u pages; %llu missing, FP rate %.4f\n",
          f.info.num_fingerprints, f.info.num_unique, f.info.num_pages, (unsigned long long)missing,
          (double)fp / n);
   rf_amd_image_free(&f);
   rf_amd_engine_destroy(e);
   free(h);
   free(fv);
   return missing == 0 && fp < n / 20 ? 0 : 1;
}
