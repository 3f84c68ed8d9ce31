// gq_host.h — internals shared by the library's translation units (gq_pileup.hip,
// gq_somatic.hip): error reporting, run counters, device buffers, the context and
// resident read-set handles, tile planning.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/gqpileup.h"
#include "gq_kernels.h"

namespace gq {

gq_status set_err(gq_status s, const char *fmt, ...);  // thread-local message for gq_last_error

#define HIP_TRY(expr)                                                                         \
  do {                                                                                        \
    hipError_t _e = (expr);                                                                   \
    if (_e != hipSuccess)                                                                     \
      return set_err(GQ_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, __LINE__); \
  } while (0)

constexpr int kBlock = 256;
constexpr int kGermT = 1024;  // loci per germline tile
constexpr int kCountT = 512;  // loci per counts tile
constexpr int kStageBytes = 40 * 1024;
constexpr size_t kSeqPad = 2048;  // zeroed tail of the uploaded sequence pool  // LDS staging of a read batch's sequence bytes

struct Counters {  // device-side run counters (one allocation, zeroed per call)
  unsigned long long n_rec;
  unsigned long long n_complex;
  unsigned long long visited;
  unsigned long long ambiguous;
  unsigned long long ties;
  unsigned long long pool_used;
  int err;
  int pad;
  long long err_pos;
  // per-tile run counters of germline_tile, spread over kSpread addresses (summed on the host)
  unsigned long long spread[3][64];
  unsigned long long prof[8];  // diagnostic phase clocks (GQ_ABLATE=32 builds only)
};
constexpr int kSpread = 64;

// Wave-aggregated reservation of `n` slots on a global counter.
__device__ __forceinline__ unsigned long long wave_reserve(unsigned long long *ctr, unsigned n) {
  if (__ballot(n != 0) == 0) return 0;  // nothing to reserve in this wave (the common case)
  const int lane = threadIdx.x & 63;
  // inclusive scan of n across the wave
  unsigned x = n;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    unsigned y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  const unsigned total = __shfl(x, 63, 64);
  unsigned long long base = 0;
  if (lane == 63 && total) base = atomicAdd(ctr, (unsigned long long)total);
  base = __shfl(base, 63, 64);
  return base + (x - n);
}

struct Plan {
  int64_t n_tiles = 0;
  int64_t n_loci = 0;
};

}  // namespace gq

// ==========================================================================================
// Host side: context, resident read sets
// ==========================================================================================
namespace gq {
struct DevBuf {
  void *p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= n) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    size_t want = std::max(bytes, (size_t)256);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) n = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};
}  // namespace gq

struct gq_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev[6] = {};
  gq_timings timings{};
  int germ_tile = gq::kGermT;
  gq::DevBuf ranges, tiles, recs, recs_sorted, keys, keys_sorted, idx, idx_sorted, cplx, pool, counters, sort_tmp, image, tiles2, srecs;
  gq::DevBuf c_depth, c_pos, c_base, c_indel, c_ref, c_rb, c_amb;
};

struct gq_dev_reads {
  gq_ctx *ctx = nullptr;
  gq::DevReads d{};
  std::vector<int64_t> contig_read_begin;  // host copy
  std::vector<void *> owned;               // device allocations owned by this handle
  int64_t seq_bytes = 0;
};

namespace gq {
// Loci ranges -> locus tiles of T loci with each tile's read window in `rd`, written to `tiles`.
gq_status plan(gq_ctx *c, const gq_dev_reads *rd, const gq_loci *loci, int T, Plan &pl, DevBuf &tiles);
gq_status check_device_error(gq_ctx *c, const Counters &h);
}  // namespace gq

