/*
 * rf_oracle.c -- CPU restatement of SplinterDB's routing filter (TEST INFRASTRUCTURE ONLY).
 *
 * See rf_oracle.h for scope and pinning. Every function cites the reference file:line it
 * restates (reference = vmware/splinterdb). Nothing here is shipped or called by the
 * product path; the product is the HIP engine in splinterdb_amd/csrc/.
 */
#include "rf_oracle.h"

#include <errno.h>
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define RFO_FPS_PER_PAGE 4096 /* ROUTING_FPS_PER_PAGE, src/routing_filter.c:26 */

/* ------------------------------------------------------------------------------------
 * XXH32 -- restated from the published xxHash algorithm (libxxhash 0.8.x). The reference
 * calls it as platform_hash32 (src/platform_linux/platform_hash.h:23) with seed 42
 * (src/splinterdb.c:276, tests/functional/test.h:286).
 * ---------------------------------------------------------------------------------- */
#define XP1 2654435761U
#define XP2 2246822519U
#define XP3 3266489917U
#define XP4 668265263U
#define XP5 374761393U

static inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static inline uint32_t rd32(const uint8_t *p)
{
   uint32_t v;
   memcpy(&v, p, 4);
   return v;
}
static inline uint32_t xround(uint32_t acc, uint32_t in)
{
   acc += in * XP2;
   acc = rotl32(acc, 13);
   return acc * XP1;
}

uint32_t rfo_xxh32(const void *input, size_t len, uint32_t seed)
{
   const uint8_t *p = (const uint8_t *)input;
   const uint8_t *end = p + len;
   uint32_t h;
   if (len >= 16) {
      const uint8_t *limit = end - 15;
      uint32_t v1 = seed + XP1 + XP2, v2 = seed + XP2, v3 = seed, v4 = seed - XP1;
      do {
         v1 = xround(v1, rd32(p));
         v2 = xround(v2, rd32(p + 4));
         v3 = xround(v3, rd32(p + 8));
         v4 = xround(v4, rd32(p + 12));
         p += 16;
      } while (p < limit);
      h = rotl32(v1, 1) + rotl32(v2, 7) + rotl32(v3, 12) + rotl32(v4, 18);
   } else {
      h = seed + XP5;
   }
   h += (uint32_t)len;
   size_t rem = len & 15;
   while (rem >= 4) {
      h += rd32(p) * XP3;
      h = rotl32(h, 17) * XP4;
      p += 4;
      rem -= 4;
   }
   while (rem > 0) {
      h += (*p++) * XP5;
      h = rotl32(h, 11) * XP1;
      rem--;
   }
   h ^= h >> 15;
   h *= XP2;
   h ^= h >> 13;
   h *= XP3;
   h ^= h >> 16;
   return h;
}

void rfo_hash_fixed(const uint8_t *keys, uint64_t n, uint32_t key_len, uint32_t seed,
                    uint32_t *out)
{
   for (uint64_t i = 0; i < n; i++) {
      out[i] = rfo_xxh32(keys + i * (uint64_t)key_len, key_len, seed);
   }
}

void rfo_hash_var(const uint8_t *bytes, const uint64_t *offs, uint64_t n, uint32_t seed,
                  uint32_t *out)
{
   for (uint64_t i = 0; i < n; i++) {
      out[i] = rfo_xxh32(bytes + offs[i], (size_t)(offs[i + 1] - offs[i]), seed);
   }
}

/* ------------------------------------------------------------------------------------
 * PackedArray -- src/PackedArray.c. Items are packed LSB-first into little-endian u32
 * words; pack preserves every bit that is not an item bit (the tail-word read-modify-
 * write at src/PackedArray.c:249-253); bitsPerItem == 0 is a no-op (the dispatch switch
 * at :391-425 has no case 0). Restated over a byte stream so unaligned block starts
 * (the reference casts char* cursors to uint32*) behave identically on little-endian.
 * ---------------------------------------------------------------------------------- */
/* nbits <= 32: the item spans at most 5 bytes from bitpos>>3; only those bytes are touched */
static inline void bs_set(uint8_t *base, uint64_t bitpos, uint32_t val, uint32_t nbits)
{
   uint8_t *p = base + (bitpos >> 3);
   uint32_t sh = (uint32_t)(bitpos & 7);
   uint32_t nbytes = (sh + nbits + 7) >> 3;
   uint64_t w = 0;
   for (uint32_t i = 0; i < nbytes; i++) {
      w |= (uint64_t)p[i] << (8 * i);
   }
   uint64_t m = ((1ULL << nbits) - 1) << sh;
   w = (w & ~m) | (((uint64_t)val << sh) & m);
   for (uint32_t i = 0; i < nbytes; i++) {
      p[i] = (uint8_t)(w >> (8 * i));
   }
}

static inline uint32_t bs_get(const uint8_t *base, uint64_t bitpos, uint32_t nbits)
{
   const uint8_t *p = base + (bitpos >> 3);
   uint32_t sh = (uint32_t)(bitpos & 7);
   uint32_t nbytes = (sh + nbits + 7) >> 3;
   uint64_t w = 0;
   for (uint32_t i = 0; i < nbytes; i++) {
      w |= (uint64_t)p[i] << (8 * i);
   }
   return (uint32_t)((w >> sh) & ((1ULL << nbits) - 1));
}

/* __PackedArray_pack_N, src/PackedArray.c:205-254 */
void rfo_pack(uint32_t *a, uint32_t offset, const uint32_t *in, uint32_t count, uint32_t bits)
{
   if (bits == 0 || bits > 32) {
      return;
   }
   uint32_t mask = (uint32_t)((1ULL << bits) - 1);
   for (uint32_t i = 0; i < count; i++) {
      bs_set((uint8_t *)a, ((uint64_t)offset + i) * bits, in[i] & mask, bits);
   }
}

/* __PackedArray_unpack_N, src/PackedArray.c:256-299 */
void rfo_unpack(const uint32_t *a, uint32_t offset, uint32_t *out, uint32_t count,
                uint32_t bits)
{
   if (bits == 0 || bits > 32) {
      return;
   }
   for (uint32_t i = 0; i < count; i++) {
      out[i] = bs_get((const uint8_t *)a, ((uint64_t)offset + i) * bits, bits);
   }
}

/* PackedArray_get, src/PackedArray.c:505-538 (bitsPerItem 0 yields 0: mask is 0) */
uint32_t rfo_get(const uint32_t *a, uint32_t offset, uint32_t bits)
{
   if (bits == 0 || bits > 32) {
      return 0;
   }
   return bs_get((const uint8_t *)a, (uint64_t)offset * bits, bits);
}

/* ------------------------------------------------------------------------------------
 * RadixSort -- src/routing_filter.c:54-131. LSD, ceil(fp_size/8) byte passes, all
 * histograms in one pass, scatter ping-pong between pData and pTemp. Returns the buffer
 * that holds the sorted result.
 * ---------------------------------------------------------------------------------- */
static uint32_t *radix_sort(uint32_t *pData, uint32_t *mBuf, uint32_t *pTemp, uint32_t count,
                            uint32_t fp_size)
{
   uint32_t *mIndex[4];
   if (fp_size == 0) {
      fp_size = 1;
   }
   uint32_t rounds = (fp_size + 7) / 8;
   for (uint32_t i = 0; i < 4; i++) {
      mIndex[i] = &mBuf[i * 256];
   }
   memset(mBuf, 0, 4 * 256 * sizeof(uint32_t));
   for (uint32_t i = 0; i < count; i++) {
      uint32_t u = pData[i];
      for (uint32_t j = 0; j < rounds; j++) {
         mIndex[j][(u >> (8 * j)) & 0xff]++;
      }
   }
   for (uint32_t j = 0; j < rounds; j++) {
      uint32_t n = 0;
      for (uint32_t i = 0; i < 256; i++) {
         uint32_t m = mIndex[j][i];
         mIndex[j][i] = n;
         n += m;
      }
   }
   uint32_t *pDst = pTemp, *pSrc = pData, *pTmp;
   for (uint32_t j = 0; j < rounds; j++) {
      for (uint32_t i = 0; i < count; i++) {
         uint32_t u = pSrc[i];
         uint32_t c = (u >> (8 * j)) & 0xff;
         pDst[mIndex[j][c]++] = u;
      }
      pTmp = pSrc;
      pSrc = pDst;
      pDst = pTmp;
   }
   return pSrc;
}

/* ------------------------------------------------------------------------------------
 * Geometry shared by add / lookup / estimate (src/routing_filter.c:357-366, 374-387,
 * 1014-1028).
 * ---------------------------------------------------------------------------------- */
static inline uint32_t log_num_buckets(const rfo_config *cfg, uint32_t num_fp)
{
   uint32_t l = 31 - (uint32_t)__builtin_clz(num_fp);
   return l < cfg->log_index_size ? cfg->log_index_size : l;
}

static inline uint64_t slots_per_extent(const rfo_config *cfg)
{
   return (uint64_t)cfg->pages_per_extent * cfg->page_size / sizeof(uint64_t);
}

/* routing_get_bucket_counts, src/routing_filter.c:281-306 (u64 words read LE) */
void rfo_bucket_counts(const rfo_config *cfg, const uint8_t *hdr, uint32_t *count)
{
   uint32_t index_size = 1u << cfg->log_index_size;
   const uint8_t *cursor = hdr + 2;
   uint64_t start = 0, end, word;
   memcpy(&word, cursor, 8);
   cursor += 8;
   memset(count, 0, index_size * sizeof(uint32_t));
   for (uint32_t i = 0; i < index_size; i++) {
      while (word == 0) {
         count[i] += 64 - start;
         start = 0;
         memcpy(&word, cursor, 8);
         cursor += 8;
      }
      end = __builtin_ffsll(word) - 1;
      word &= word - 1;
      count[i] += end - start;
      start = end + 1;
   }
}

/* routing_get_bucket_bounds, src/routing_filter.c:230-279 (u32 words read LE) */
static void bucket_bounds(const uint8_t *encoding, uint64_t len, uint64_t bucket_offset,
                          uint64_t *start, uint64_t *end)
{
   uint32_t word = 0, encoding_word = 0;
   uint64_t bucket = 0, bucket_pop = 0, bit_offset = 0;
   if (bucket_offset == 0) {
      *start = 0;
      word = 0;
      encoding_word = rd32(encoding);
      while (encoding_word == 0) {
         word++;
         encoding_word = rd32(encoding + 4 * word);
      }
      bit_offset = __builtin_ffs(encoding_word) - 1;
      *end = 32 * (uint64_t)word + bit_offset;
   } else {
      bucket_pop = __builtin_popcount(rd32(encoding));
      while (4 * (uint64_t)word < len && bucket + bucket_pop < bucket_offset) {
         bucket += bucket_pop;
         word++;
         bucket_pop = __builtin_popcount(rd32(encoding + 4 * word));
      }
      encoding_word = rd32(encoding + 4 * word);
      while (bucket < bucket_offset - 1) {
         encoding_word &= encoding_word - 1;
         bucket++;
      }
      bit_offset = __builtin_ffs(encoding_word) - 1;
      *start = 32 * (uint64_t)word + bit_offset - bucket_offset + 1;
      encoding_word &= encoding_word - 1;
      while (encoding_word == 0) {
         word++;
         encoding_word = rd32(encoding + 4 * word);
      }
      bit_offset = __builtin_ffs(encoding_word) - 1;
      *end = 32 * (uint64_t)word + bit_offset - bucket_offset;
   }
}

/* exported for tests/test_ref_pinning.py, which fuzzes them against the reference's own
 * static RadixSort / routing_get_bucket_bounds (oracle/ref_static.c) */
uint32_t *rfo_radix_sort(uint32_t *pData, uint32_t *pTemp, uint32_t count, uint32_t fp_size)
{
   uint32_t mBuf[4 * 256];
   return radix_sort(pData, mBuf, pTemp, count, fp_size);
}

void rfo_bucket_bounds(const uint8_t *encoding, uint64_t len, uint64_t bucket_offset, uint64_t *start,
                       uint64_t *end)
{
   bucket_bounds(encoding, len, bucket_offset, start, end);
}

static int ensure_pages(const rfo_config *cfg, rfo_filter *f, uint32_t need)
{
   if (need <= f->pages_cap) {
      return 0;
   }
   uint32_t cap = f->pages_cap ? f->pages_cap : 16;
   while (cap < need) {
      cap *= 2;
   }
   /* +1 page of zero slack so u32/u64 encoding reads near the last page stay in bounds */
   uint8_t *np = (uint8_t *)realloc(f->pages, ((size_t)cap + 1) * cfg->page_size);
   if (np == NULL) {
      return ENOMEM;
   }
   memset(np + (size_t)f->pages_cap * cfg->page_size, 0,
          ((size_t)cap + 1 - f->pages_cap) * cfg->page_size);
   f->pages = np;
   f->pages_cap = cap;
   return 0;
}

void rfo_filter_release(rfo_filter *f)
{
   if (f == NULL) {
      return;
   }
   free(f->slots);
   free(f->pages);
   memset(f, 0, sizeof(*f));
}

/* ------------------------------------------------------------------------------------
 * routing_filter_add -- src/routing_filter.c:337-656.
 *
 * Deviations (all are undefined behaviour or crashes in the reference, rejected here
 * with EINVAL instead): total fingerprints == 0 (__builtin_clz(0), :374); more indices
 * than one extent of slots (index_page[] overflow, :441-449, :613-617); an index with
 * more than ROUTING_FPS_PER_PAGE entries (fp_buffer overflow, :596); a block larger
 * than a page (:603-610 writes past the page); fp_size + value_size > 32 (asserted,
 * :389); a value narrower than the old filter's (negative shift at :540).
 * ---------------------------------------------------------------------------------- */
int rfo_filter_add(const rfo_config *cfg, const rfo_filter *old_filter, rfo_filter *filter,
                   uint32_t *new_fp_arr, uint64_t num_new_fp, uint16_t value)
{
   memset(filter, 0, sizeof(*filter));
   const int has_old = old_filter != NULL && old_filter->slots != NULL;
   const uint32_t index_size = 1u << cfg->log_index_size;
   const uint32_t page_size = cfg->page_size;

   uint32_t old_num_indices = 1, old_value_size = 0, old_value_mask = 0, old_rvs = 0;
   if (has_old) {
      uint32_t old_lnb = log_num_buckets(cfg, old_filter->num_fingerprints);
      old_num_indices = 1u << (old_lnb - cfg->log_index_size);
      uint32_t old_rem = cfg->fingerprint_size - old_lnb;
      old_value_size = old_filter->value_size;
      old_value_mask = (uint32_t)((1ULL << old_value_size) - 1);
      old_rvs = old_value_size + old_rem;
      if (cfg->fingerprint_size + old_value_size > 32) {
         return EINVAL;
      }
   }

   uint32_t num_fp = (uint32_t)(num_new_fp + (old_filter ? old_filter->num_fingerprints : 0));
   if (num_fp == 0) {
      return EINVAL;
   }
   filter->num_fingerprints = num_fp;
   filter->num_unique = 0;
   uint32_t lnb = log_num_buckets(cfg, num_fp);
   if (lnb > cfg->fingerprint_size) {
      return EINVAL;
   }
   uint32_t num_indices = 1u << (lnb - cfg->log_index_size);
   if (num_indices > slots_per_extent(cfg)) {
      return EINVAL;
   }
   uint32_t remainder_size = cfg->fingerprint_size - lnb;
   uint32_t value_size = value == 0 ? 0 : 32 - (uint32_t)__builtin_clz(value);
   filter->value_size = value_size;
   filter->num_indices = num_indices;
   uint32_t rvs = value_size + remainder_size;
   uint32_t rv_mask = (uint32_t)((1ULL << rvs) - 1);
   uint32_t irvs = rvs + cfg->log_index_size;
   uint32_t new_indices_per_old_index = num_indices / old_num_indices;
   if (cfg->fingerprint_size + value_size > 32) {
      return EINVAL;
   }
   if (has_old && value_size < old_value_size) {
      return EINVAL;
   }

   /* scratch: temp | index_count | old_count | matrix | fp_buffer | old_fp_buffer | enc */
   size_t enc_bytes = (RFO_FPS_PER_PAGE + index_size) / 8 + 64;
   uint32_t *temp = (uint32_t *)calloc(num_new_fp + num_indices + index_size + 1024 +
                                          2 * RFO_FPS_PER_PAGE + 64,
                                       sizeof(uint32_t));
   uint8_t *encoding_buffer = (uint8_t *)malloc(enc_bytes);
   filter->slots = (uint64_t *)calloc(slots_per_extent(cfg), sizeof(uint64_t));
   if (temp == NULL || encoding_buffer == NULL || filter->slots == NULL) {
      free(temp);
      free(encoding_buffer);
      rfo_filter_release(filter);
      return ENOMEM;
   }
   uint32_t *index_count = temp + num_new_fp;
   uint32_t *old_count = index_count + num_indices;
   uint32_t *matrix = old_count + index_size;
   uint32_t *fp_buffer = matrix + 1024;
   uint32_t *old_fp_buffer = fp_buffer + RFO_FPS_PER_PAGE;
   memset(encoding_buffer, 0xff, enc_bytes);

   int rc = 0;
   uint32_t page_no = 0;
   if ((rc = ensure_pages(cfg, filter, 1)) != 0) {
      goto fail;
   }
   filter->num_pages = 1;
   uint64_t cursor = 0; /* byte offset within the current page */
   uint64_t bytes_remaining_on_page = page_size;

   for (uint64_t i = 0; i < num_new_fp; i++) {
      new_fp_arr[i] >>= 32 - cfg->fingerprint_size;
   }
   uint32_t *fp_arr = new_fp_arr;
   if (num_new_fp > 0) {
      fp_arr = radix_sort(new_fp_arr, matrix, temp, (uint32_t)num_new_fp,
                          cfg->fingerprint_size);
   }
   for (uint64_t i = 0; i < num_new_fp; i++) {
      fp_arr[i] <<= value_size;
      fp_arr[i] |= value;
   }
   /* dedupe, :471-482 */
   uint32_t dst = 0;
   uint64_t num_new_unique_fp = num_new_fp;
   for (uint64_t src = 0; src != num_new_fp; src++) {
      fp_arr[dst] = fp_arr[src];
      if (dst == 0 || fp_arr[dst] != fp_arr[dst - 1]) {
         dst++;
      } else {
         num_new_unique_fp--;
      }
   }
   /* per-index counts, :484-494 */
   uint32_t fp_no = 0;
   for (uint32_t index_no = 0; index_no < num_indices; index_no++) {
      uint32_t index_start = fp_no;
      while (fp_no < num_new_unique_fp &&
             (irvs == 32 ? 0 : fp_arr[fp_no] >> irvs) == index_no) {
         fp_no++;
      }
      index_count[index_no] = fp_no - index_start;
   }

   fp_no = 0;
   for (uint32_t old_index_no = 0; old_index_no < old_num_indices; old_index_no++) {
      uint32_t old_index_count = 0;
      uint32_t *old_src_fp = old_fp_buffer;
      uint32_t *dst_fp = fp_buffer;
      uint32_t index_bucket_start = old_index_no * index_size;
      if (has_old) {
         /* routing_get_header, :178-198 (relocatable slot = page_no*page_size + off) */
         const uint8_t *old_hdr = old_filter->pages + old_filter->slots[old_index_no];
         uint32_t nrem = (uint32_t)old_hdr[0] | ((uint32_t)old_hdr[1] << 8);
         uint64_t header_length = (nrem + index_size - 1) / 8 + 4 + 2;
         const uint8_t *old_block_start = old_hdr + header_length;
         old_index_count = nrem;
         rfo_bucket_counts(cfg, old_hdr, old_count);
         if (old_index_count != 0) {
            if (old_index_count > RFO_FPS_PER_PAGE) {
               rc = EINVAL;
               goto fail;
            }
            rfo_unpack((const uint32_t *)old_block_start, 0, old_src_fp, old_index_count,
                       old_rvs);
            uint32_t old_fp_no = 0;
            for (uint32_t bucket_off = 0; bucket_off < index_size; bucket_off++) {
               uint32_t bucket = index_bucket_start + bucket_off;
               for (uint32_t i = 0; i < old_count[bucket_off]; i++) {
                  old_src_fp[old_fp_no++] |= old_rvs >= 32 ? 0 : bucket << old_rvs;
               }
            }
            if (old_value_size != value_size) {
               for (old_fp_no = 0; old_fp_no < old_index_count; old_fp_no++) {
                  uint32_t old_value = old_src_fp[old_fp_no] & old_value_mask;
                  old_src_fp[old_fp_no] -= old_value;
                  old_src_fp[old_fp_no] <<= (value_size - old_value_size);
                  old_src_fp[old_fp_no] |= old_value;
               }
            }
         }
      }
      uint32_t old_fps_added = 0;
      for (uint32_t index_off = 0; index_off < new_indices_per_old_index; index_off++) {
         uint32_t *new_src_fp = &fp_arr[fp_no];
         uint32_t index_no = old_index_no * new_indices_per_old_index + index_off;
         uint32_t last_bucket = index_no * index_size;
         uint32_t fps_added = 0, new_fps_added = 0;
         uint32_t end_bucket = (index_no + 1) * index_size;
         uint32_t new_index_count = index_count[index_no];
         uint64_t header_bit = 0;
         uint32_t last_fp_added = UINT32_MAX;
         /* 2-way merge, old first on ties, :559-597 */
         while (new_fps_added < new_index_count || old_fps_added < old_index_count) {
            uint32_t fp;
            int is_old = (new_fps_added == new_index_count) ||
                         ((old_fps_added != old_index_count) &&
                          (old_src_fp[old_fps_added] <= new_src_fp[new_fps_added]));
            if (is_old) {
               fp = old_src_fp[old_fps_added++];
            } else {
               fp = new_src_fp[new_fps_added++];
            }
            if (last_fp_added >> value_size != fp >> value_size) {
               filter->num_unique++;
            }
            uint32_t bucket = rvs >= 32 ? 0 : fp >> rvs;
            if (bucket >= end_bucket) {
               old_fps_added--;
               break;
            }
            header_bit += bucket - last_bucket;
            last_bucket = bucket;
            encoding_buffer[header_bit >> 3] &= (uint8_t)~(1u << (header_bit & 7));
            header_bit++;
            last_fp_added = fp;
            if (fps_added >= RFO_FPS_PER_PAGE) {
               rc = EINVAL;
               goto fail;
            }
            dst_fp[fps_added++] = fp & rv_mask;
         }

         /* block sizes, :599-602 (u32 truncation gives 3 when fps_added*rvs == 0) */
         uint32_t remainder_block_size = (uint32_t)(((uint64_t)fps_added * rvs - 1) / 8 + 4);
         uint64_t encoding_size = ((uint64_t)fps_added + index_size - 1) / 8 + 4;
         uint32_t header_size = (uint32_t)encoding_size + 2;
         if ((uint64_t)header_size + remainder_block_size > page_size) {
            rc = EINVAL;
            goto fail;
         }
         /* greedy page placement, :603-610 */
         if (header_size + remainder_block_size > bytes_remaining_on_page) {
            page_no++;
            if ((rc = ensure_pages(cfg, filter, page_no + 1)) != 0) {
               goto fail;
            }
            filter->num_pages = page_no + 1;
            bytes_remaining_on_page = page_size;
            cursor = 0;
         }
         /* index slot, :612-620 */
         filter->slots[index_no] = (uint64_t)page_no * page_size + cursor;
         uint8_t *hdr = filter->pages + (size_t)page_no * page_size + cursor;
         hdr[0] = (uint8_t)(fps_added & 0xff);
         hdr[1] = (uint8_t)(fps_added >> 8);
         memmove(hdr + 2, encoding_buffer, encoding_size);
         memset(encoding_buffer, 0xff, encoding_size);
         cursor += header_size;
         if (fps_added != 0) {
            rfo_pack((uint32_t *)(filter->pages + (size_t)page_no * page_size + cursor), 0,
                     fp_buffer, fps_added, rvs);
         }
         fp_no += index_count[index_no];
         cursor += remainder_block_size;
         bytes_remaining_on_page -= header_size + remainder_block_size;
      }
   }
   free(temp);
   free(encoding_buffer);
   return 0;

fail:
   free(temp);
   free(encoding_buffer);
   rfo_filter_release(filter);
   return rc;
}

/* ------------------------------------------------------------------------------------
 * routing_filter_lookup -- src/routing_filter.c:985-1073, with the key already hashed
 * (data_key_hash at :1011). A NULL filter (addr == 0) finds nothing (:1003-1006).
 * ---------------------------------------------------------------------------------- */
uint64_t rfo_filter_lookup_hash(const rfo_config *cfg, const rfo_filter *filter, uint32_t hash)
{
   if (filter == NULL || filter->slots == NULL) {
      return 0;
   }
   uint32_t index_size = 1u << cfg->log_index_size;
   uint32_t fp = hash >> (32 - cfg->fingerprint_size);
   uint32_t value_size = filter->value_size;
   uint32_t lnb = log_num_buckets(cfg, filter->num_fingerprints);
   uint32_t remainder_size = cfg->fingerprint_size - lnb;
   uint32_t rvs = remainder_size + value_size;
   uint32_t bucket = rvs >= 32 ? 0 : (fp << value_size) >> rvs;
   uint32_t bucket_off = bucket % index_size;
   uint32_t irvs = rvs + cfg->log_index_size;
   uint32_t remainder_mask = (uint32_t)((1ULL << remainder_size) - 1);
   uint32_t index = irvs >= 32 ? 0 : (fp << value_size) >> irvs;
   uint32_t remainder = fp & remainder_mask;

   const uint8_t *hdr = filter->pages + filter->slots[index];
   uint32_t nrem = (uint32_t)hdr[0] | ((uint32_t)hdr[1] << 8);
   uint64_t encoding_size = (nrem + (uint64_t)index_size - 1) / 8 + 4;
   uint64_t header_length = encoding_size + 2;
   uint64_t start, end;
   bucket_bounds(hdr + 2, header_length, bucket_off, &start, &end);
   const uint8_t *block = hdr + header_length;
   if (start == end) {
      return 0;
   }
   uint64_t found = 0;
   uint32_t value_mask = (uint32_t)((1ULL << value_size) - 1);
   for (uint32_t i = 0; i < end - start; i++) {
      uint32_t pos = (uint32_t)(end - i - 1);
      uint32_t rv = rfo_get((const uint32_t *)block, pos, rvs);
      if ((rv >> value_size) == remainder) {
         uint32_t found_value = rv & value_mask;
         if (found_value < 64) { /* platform_assert(found_value < 64), :1064 */
            found |= 1ULL << found_value;
         }
      }
   }
   return found;
}

void rfo_filter_lookup_hashes(const rfo_config *cfg, const rfo_filter *f, const uint32_t *hashes,
                              uint64_t n, uint64_t *found)
{
   for (uint64_t i = 0; i < n; i++) {
      found[i] = rfo_filter_lookup_hash(cfg, f, hashes[i]);
   }
}

/* ------------------------------------------------------------------------------------
 * routing_filter_estimate_unique_fp -- src/routing_filter.c:702-848. Decodes the first
 * 1/16 of each filter's indices, dedupes fingerprints (value bits dropped) per filter,
 * counts the distinct union with a k-way merge, and scales by 16.
 * ---------------------------------------------------------------------------------- */
int rfo_estimate_unique_fp(const rfo_config *cfg, const rfo_filter *filters,
                           uint64_t num_filters, uint32_t *num_unique_fp)
{
   if (num_unique_fp == NULL) {
      return EINVAL;
   }
   *num_unique_fp = 0;
   if (num_filters > 32) {
      return EINVAL;
   }
   uint32_t index_size = 1u << cfg->log_index_size;
   uint32_t total_num_fp = 0;
   for (uint64_t i = 0; i != num_filters; i++) {
      total_num_fp += filters[i].num_fingerprints;
   }
   uint32_t buffer_size = total_num_fp / 12;
   uint32_t *local = (uint32_t *)calloc((size_t)buffer_size + index_size, sizeof(uint32_t));
   if (local == NULL) {
      return ENOMEM;
   }
   uint32_t *fp_arr = local;
   uint32_t *count = local + buffer_size;
   uint32_t src_fp_no = 0, dst_fp_no = 0;
   uint32_t fp_start[33] = {0};
   for (uint64_t i = 0; i != num_filters; i++) {
      const rfo_filter *f = &filters[i];
      if (f->slots == NULL) {
         fp_start[i + 1] = dst_fp_no;
         continue;
      }
      uint32_t lnb = log_num_buckets(cfg, f->num_fingerprints);
      uint32_t num_indices = 1u << (lnb - cfg->log_index_size);
      uint32_t remainder_size = cfg->fingerprint_size - lnb;
      uint32_t value_size = f->value_size;
      uint32_t rvs = value_size + remainder_size;
      if (num_indices >= 16) {
         num_indices /= 16;
         for (uint32_t index_no = 0; index_no < num_indices; index_no++) {
            const uint8_t *hdr = f->pages + f->slots[index_no];
            uint32_t index_count = (uint32_t)hdr[0] | ((uint32_t)hdr[1] << 8);
            uint64_t header_length = (index_count + index_size - 1) / 8 + 4 + 2;
            const uint8_t *block_start = hdr + header_length;
            rfo_bucket_counts(cfg, hdr, count);
            uint32_t index_bucket_start = index_no * index_size;
            if (src_fp_no + index_count > buffer_size) {
               free(local);
               return EINVAL; /* platform_assert at :777 */
            }
            if (index_count != 0) {
               rfo_unpack((const uint32_t *)block_start, 0, &fp_arr[src_fp_no], index_count, rvs);
               uint32_t last_fp = UINT32_MAX;
               for (uint32_t bucket_off = 0; bucket_off < index_size; bucket_off++) {
                  uint32_t bucket = index_bucket_start + bucket_off;
                  for (uint32_t k = 0; k < count[bucket_off]; k++) {
                     fp_arr[src_fp_no] |= rvs >= 32 ? 0 : bucket << rvs;
                     fp_arr[src_fp_no] >>= value_size;
                     if (fp_arr[src_fp_no] == last_fp) {
                        src_fp_no++;
                     } else {
                        last_fp = fp_arr[src_fp_no];
                        fp_arr[dst_fp_no++] = fp_arr[src_fp_no++];
                     }
                  }
               }
            }
         }
      }
      fp_start[i + 1] = dst_fp_no;
   }
   uint32_t idx[33];
   memcpy(idx, fp_start, sizeof(idx));
   uint32_t num_unique = 0;
   for (;;) {
      uint32_t min_fp = UINT32_MAX;
      for (uint64_t i = 0; i < num_filters; i++) {
         if (idx[i] != fp_start[i + 1] && fp_arr[idx[i]] < min_fp) {
            min_fp = fp_arr[idx[i]];
         }
      }
      if (min_fp == UINT32_MAX) {
         break;
      }
      for (uint64_t i = 0; i < num_filters; i++) {
         if (idx[i] != fp_start[i + 1] && fp_arr[idx[i]] == min_fp) {
            idx[i]++;
         }
      }
      num_unique++;
   }
   free(local);
   *num_unique_fp = num_unique * 16;
   return 0;
}

/* routing_filter_estimate_unique_keys_from_count, src/routing_filter.c:1119-1139, evaluated as
 * the reference's release build evaluates it (-O3 -ffast-math, Makefile:89,123-124): GCC
 * reassociates the sum into two fused multiply-adds,
 *   (fma(1/U - 1/s, 1/2, (1/s^2 - 1/U^2) * (1/12)) + fma(1/U^4 - 1/s^4, 1/120, log U)) - log s,
 * and converts U * that through a 64-bit truncation. The order matters where the exact value
 * is an integer: num_unique = 1 gives exactly 1 (H_U - H_{U-1} = 1/U) -- 1 in the reference's
 * build, 0 in the source order. Checked against the reference for every fingerprint size 8-32
 * (tests/test_ref_pinning.py). */
uint32_t rfo_estimate_unique_keys_from_count(const rfo_config *cfg, uint64_t num_unique)
{
   const double U = (double)(1UL << cfg->fingerprint_size);
   const double s = U - (double)num_unique;
   const double U2 = U * U, s2 = s * s;
   const double lU = log(U), ls = log(s);
   const double a = fma(1.0 / U - 1.0 / s, 0.5, (1.0 / s2 - 1.0 / U2) * (1.0 / 12.0));
   const double b = fma(1.0 / (U2 * U2) - 1.0 / (s2 * s2), 1.0 / 120.0, lU);
   return (uint32_t)(int64_t)(U * ((a + b) - ls));
}

/*
 * routing_filter_space_use_bytes (src/routing_filter.c:1149-1153) = mini_space_use_bytes
 * of the filter's unkeyed mini allocator (src/mini_allocator.c:1094-1101): one meta page
 * plus every extent it handed out (the index extent, then ceil(data_pages/32) extents).
 */
uint64_t rfo_space_use_bytes(const rfo_config *cfg, const rfo_filter *f)
{
   if (f == NULL || f->slots == NULL) {
      return 0;
   }
   uint64_t extent = (uint64_t)cfg->page_size * cfg->pages_per_extent;
   uint64_t data_extents = (f->num_pages + cfg->pages_per_extent - 1) / cfg->pages_per_extent;
   return cfg->page_size + extent * (1 + data_extents);
}

rfo_filter *rfo_filter_new(void) { return (rfo_filter *)calloc(1, sizeof(rfo_filter)); }
void rfo_filter_delete(rfo_filter *f)
{
   rfo_filter_release(f);
   free(f);
}

/* ------------------------------------------------------------------------------------
 * Multi-threaded CPU baseline: one routing_filter_add per task, tasks pulled by worker
 * threads -- the reference's concurrency model (TASK_TYPE_NORMAL, src/trunk.c:3932).
 * ---------------------------------------------------------------------------------- */
typedef struct bench_ctx {
   const rfo_config *cfg;
   const uint8_t *keys;
   uint32_t key_len;
   int hash_keys;
   const uint64_t *key_start;
   const uint32_t *key_count;
   uint32_t num_filters;
   uint16_t value;
   rfo_filter *keep;
   _Atomic uint32_t next;
   _Atomic int err;
   const uint64_t *offs; /* variable-length keys: key i = keys[offs[i] .. offs[i+1]) */
   /* probe */
   const rfo_filter *filters;
   const uint32_t *filter_id;
   uint64_t n;
   uint64_t *found;
} bench_ctx;

static double now_s(void)
{
   struct timespec ts;
   clock_gettime(CLOCK_MONOTONIC, &ts);
   return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void *build_worker(void *arg)
{
   bench_ctx *c = (bench_ctx *)arg;
   for (;;) {
      uint32_t f = atomic_fetch_add(&c->next, 1);
      if (f >= c->num_filters) {
         break;
      }
      uint32_t n = c->key_count[f];
      uint32_t *fps = (uint32_t *)malloc((size_t)n * sizeof(uint32_t) + 4);
      if (c->offs) {
         rfo_hash_var(c->keys, c->offs + c->key_start[f], n, c->cfg->seed, fps);
      } else if (c->hash_keys) {
         rfo_hash_fixed(c->keys + c->key_start[f] * c->key_len, n, c->key_len, c->cfg->seed, fps);
      } else {
         memcpy(fps, (const uint32_t *)c->keys + c->key_start[f], (size_t)n * 4);
      }
      rfo_filter tmp;
      rfo_filter *dst = c->keep ? &c->keep[f] : &tmp;
      int rc = rfo_filter_add(c->cfg, NULL, dst, fps, n, c->value);
      if (rc) {
         atomic_store(&c->err, rc);
      }
      if (!c->keep) {
         rfo_filter_release(&tmp);
      }
      free(fps);
   }
   return NULL;
}

static double bench_build(const rfo_config *cfg, const uint8_t *keys, const uint64_t *offs,
                          uint32_t key_len, int hash_keys, const uint64_t *key_start,
                          const uint32_t *key_count, uint32_t num_filters, uint16_t value,
                          int threads, rfo_filter *keep)
{
   bench_ctx c;
   memset(&c, 0, sizeof(c));
   c.offs = offs;
   c.cfg = cfg;
   c.keys = keys;
   c.key_len = key_len;
   c.hash_keys = hash_keys;
   c.key_start = key_start;
   c.key_count = key_count;
   c.num_filters = num_filters;
   c.value = value;
   c.keep = keep;
   if (threads < 1) {
      threads = 1;
   }
   pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
   double t0 = now_s();
   for (int t = 0; t < threads; t++) {
      pthread_create(&th[t], NULL, build_worker, &c);
   }
   for (int t = 0; t < threads; t++) {
      pthread_join(th[t], NULL);
   }
   double t1 = now_s();
   free(th);
   return atomic_load(&c.err) ? -1.0 : t1 - t0;
}

static void *probe_worker(void *arg)
{
   bench_ctx *c = (bench_ctx *)arg;
   const uint64_t chunk = 4096;
   for (;;) {
      uint64_t s = (uint64_t)atomic_fetch_add(&c->next, 1) * chunk;
      if (s >= c->n) {
         break;
      }
      uint64_t e = s + chunk < c->n ? s + chunk : c->n;
      for (uint64_t i = s; i < e; i++) {
         uint32_t h = c->offs ? rfo_xxh32(c->keys + c->offs[i], (size_t)(c->offs[i + 1] - c->offs[i]),
                                          c->cfg->seed)
                              : rfo_xxh32(c->keys + i * c->key_len, c->key_len, c->cfg->seed);
         c->found[i] = rfo_filter_lookup_hash(c->cfg, &c->filters[c->filter_id[i]], h);
      }
   }
   return NULL;
}

double rfo_bench_build(const rfo_config *cfg, const uint8_t *keys, uint32_t key_len,
                       int hash_keys, const uint64_t *key_start, const uint32_t *key_count,
                       uint32_t num_filters, uint16_t value, int threads, rfo_filter *keep)
{
   return bench_build(cfg, keys, NULL, key_len, hash_keys, key_start, key_count, num_filters,
                      value, threads, keep);
}

double rfo_bench_build_var(const rfo_config *cfg, const uint8_t *bytes, const uint64_t *offs,
                           const uint64_t *key_start, const uint32_t *key_count,
                           uint32_t num_filters, uint16_t value, int threads, rfo_filter *keep)
{
   return bench_build(cfg, bytes, offs, 0, 1, key_start, key_count, num_filters, value, threads,
                      keep);
}

static double bench_probe(const rfo_config *cfg, const rfo_filter *filters, const uint8_t *keys,
                          const uint64_t *offs, uint32_t key_len, const uint32_t *filter_id,
                          uint64_t n, int threads, uint64_t *found)
{
   bench_ctx c;
   memset(&c, 0, sizeof(c));
   c.offs = offs;
   c.cfg = cfg;
   c.keys = keys;
   c.key_len = key_len;
   c.filters = filters;
   c.filter_id = filter_id;
   c.n = n;
   c.found = found;
   if (threads < 1) {
      threads = 1;
   }
   pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
   double t0 = now_s();
   for (int t = 0; t < threads; t++) {
      pthread_create(&th[t], NULL, probe_worker, &c);
   }
   for (int t = 0; t < threads; t++) {
      pthread_join(th[t], NULL);
   }
   double t1 = now_s();
   free(th);
   return t1 - t0;
}

double rfo_bench_probe(const rfo_config *cfg, const rfo_filter *filters, const uint8_t *keys,
                       uint32_t key_len, const uint32_t *filter_id, uint64_t n, int threads,
                       uint64_t *found)
{
   return bench_probe(cfg, filters, keys, NULL, key_len, filter_id, n, threads, found);
}

double rfo_bench_probe_var(const rfo_config *cfg, const rfo_filter *filters, const uint8_t *bytes,
                           const uint64_t *offs, const uint32_t *filter_id, uint64_t n,
                           int threads, uint64_t *found)
{
   return bench_probe(cfg, filters, bytes, offs, 0, filter_id, n, threads, found);
}
