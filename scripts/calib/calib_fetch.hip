// calib_fetch.hip — FETCH_SIZE / WRITE_SIZE calibration for the access shapes the traffic
// tables report.  Each kernel touches every byte of a 1 GiB buffer (4x the
// 256 MiB Infinity Cache, so nothing is re-served on-die) exactly once in one access shape; the
// PMC byte counter of that launch divided into the known byte count is the shape's correction
// factor.  Run under `rocprofv3 --pmc FETCH_SIZE` and, separately, `--pmc WRITE_SIZE`
// (scripts/calib/calib.sh); the kernel names carry the shape.
//
//   stream16      16 B per lane, a wave's 1 KiB contiguous (the guide's calibrated shape: x2)
//   u64_coal_ua   8 B per lane at an unaligned offset (+3), a wave's 512 B contiguous
//                 (germline_direct / proj_fill_cells cell loads within one read's run)
//   u64_lane_ua   8 B per lane, each lane streaming its own 512 B stretch (+3), so one load
//                 instruction touches 64 different lines (germline_direct's lane-private slot
//                 walk: each lane on a different read's bytes)
//   u64_g4_ua     8 B per lane, groups of four lanes on 32 contiguous bytes (+3), 16 groups on 16
//                 different stretches (the direct kernels' group-of-four slot walk)
//   b32_rows      4 B per lane, a wave's 256 B contiguous (germline_proj's projection rows)
//   rec64_perm    a lane reads one 64-byte record (four 16-byte loads) at a permuted record
//                 index (the callers' scattered per-read record loads)
//   u16_perm      2 B per lane at a permuted 64-byte record's head (a narrow scattered field load:
//                 only 1/32 of each record's line is used, so FETCH counts whole requests)
//   wr_stream16   16 B stores per lane, contiguous (the guide's calibrated store shape: x1)
//   wr_u64        8 B stores per lane, a wave's 512 B contiguous (the fill's word stores)
// Each reading kernel folds what it loaded into one dword per thread (a vector store into a
// small sink), so nothing is dead code.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                 \
      exit(1);                                                                                  \
    }                                                                                           \
  } while (0)

constexpr size_t kBytes = size_t(1) << 30;  // 1 GiB
constexpr int kThreads = 256;

// a bijection on [0, n) for n a power of two: odd multiplier, xor-shift (records scattered
// across the buffer, each visited once)
__device__ __forceinline__ uint64_t perm(uint64_t i, uint64_t n) {
  uint64_t x = (i * 0x9E3779B97F4A7C15ull) & (n - 1);
  x ^= x >> 7;
  return (x * 0xBF58476D1CE4E5B9ull + 0x1234567ull) & (n - 1);
}

__global__ __launch_bounds__(kThreads) void stream16(const uint4 *__restrict__ a, size_t n16, uint32_t *sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < n16; i += (size_t)gridDim.x * kThreads) {
    const uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  sink[blockIdx.x * kThreads + threadIdx.x] = acc;
}

// lanes of a wave: 8 B each at +3 within the wave's 512-B chunk (the last lane's load reaches 3
// bytes into the next chunk; chunk c's first 3 bytes are read by chunk c - 1's wave)
__global__ __launch_bounds__(kThreads) void u64_coal_ua(const uint8_t *__restrict__ a, size_t nchunks, uint32_t *sink) {
  const int lane = threadIdx.x & 63;
  const size_t w0 = (blockIdx.x * (size_t)kThreads + threadIdx.x) >> 6, ws = ((size_t)gridDim.x * kThreads) >> 6;
  uint32_t acc = 0;
  for (size_t c = w0; c + 1 < nchunks; c += ws) {  // (buffer loads at any byte offset, as the product's)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(a + 512 * c), (short)0, 1024, 0x00020000);
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, 3 + 8 * lane, 0, 0);
    acc ^= v[0] ^ v[1];
  }
  sink[blockIdx.x * kThreads + threadIdx.x] = acc;
}

// each lane streams its own 512-B stretch of the wave's 32 KiB chunk, 8 B (+3) per instruction
__global__ __launch_bounds__(kThreads) void u64_lane_ua(const uint8_t *__restrict__ a, size_t nchunks, uint32_t *sink) {
  const int lane = threadIdx.x & 63;
  const size_t w0 = (blockIdx.x * (size_t)kThreads + threadIdx.x) >> 6, ws = ((size_t)gridDim.x * kThreads) >> 6;
  uint32_t acc = 0;
  for (size_t c = w0; c + 1 < nchunks; c += ws) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(a + 32768 * c), (short)0, 65536, 0x00020000);
#pragma unroll 8
    for (int i = 0; i < 64; ++i) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, 512 * lane + 3 + 8 * i, 0, 0);
      acc ^= v[0] ^ v[1];
    }
  }
  sink[blockIdx.x * kThreads + threadIdx.x] = acc;
}

// groups of four lanes: each group streams its own 2 KiB stretch of the wave's 32 KiB chunk,
// 32 contiguous bytes (+3) per instruction (germline_direct / somatic_direct's group-of-four
// slot walk: a group's lanes on one read's 32 bytes, the 16 groups on 16 reads)
__global__ __launch_bounds__(kThreads) void u64_g4_ua(const uint8_t *__restrict__ a, size_t nchunks, uint32_t *sink) {
  const int lane = threadIdx.x & 63, g = lane >> 2, gl = lane & 3;
  const size_t w0 = (blockIdx.x * (size_t)kThreads + threadIdx.x) >> 6, ws = ((size_t)gridDim.x * kThreads) >> 6;
  uint32_t acc = 0;
  for (size_t c = w0; c + 1 < nchunks; c += ws) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(a + 32768 * c), (short)0, 65536, 0x00020000);
#pragma unroll 8
    for (int i = 0; i < 64; ++i) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, 2048 * g + 32 * i + 8 * gl + 3, 0, 0);
      acc ^= v[0] ^ v[1];
    }
  }
  sink[blockIdx.x * kThreads + threadIdx.x] = acc;
}

__global__ __launch_bounds__(kThreads) void b32_rows(const uint32_t *__restrict__ a, size_t n4, uint32_t *sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < n4; i += (size_t)gridDim.x * kThreads) acc ^= a[i];
  sink[blockIdx.x * kThreads + threadIdx.x] = acc;
}

__global__ __launch_bounds__(kThreads) void rec64_perm(const uint4 *__restrict__ a, size_t nrec, uint32_t *sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < nrec; i += (size_t)gridDim.x * kThreads) {
    const uint4 *r = a + 4 * perm(i, nrec);
    const uint4 x = r[0], y = r[1], z = r[2], w = r[3];
    acc ^= x.x ^ x.y ^ x.z ^ x.w ^ y.x ^ y.y ^ y.z ^ y.w ^ z.x ^ z.y ^ z.z ^ z.w ^ w.x ^ w.y ^ w.z ^ w.w;
  }
  sink[blockIdx.x * kThreads + threadIdx.x] = acc;
}

__global__ __launch_bounds__(kThreads) void u16_perm(const uint16_t *__restrict__ a, size_t nrec, uint32_t *sink) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < nrec; i += (size_t)gridDim.x * kThreads)
    acc ^= a[32 * perm(i, nrec)];
  sink[blockIdx.x * kThreads + threadIdx.x] = acc;
}

__global__ __launch_bounds__(kThreads) void wr_stream16(uint4 *__restrict__ a, size_t n16) {
  for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < n16; i += (size_t)gridDim.x * kThreads)
    a[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

__global__ __launch_bounds__(kThreads) void wr_u64(uint2 *__restrict__ a, size_t n8) {
  for (size_t i = blockIdx.x * (size_t)kThreads + threadIdx.x; i < n8; i += (size_t)gridDim.x * kThreads)
    a[i] = make_uint2((uint32_t)i, 7u);
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 3;
  uint8_t *buf;
  uint32_t *sink;
  const int grid = 256 * 8;  // 8 workgroups per CU
  CK(hipMalloc(&buf, kBytes + 4096));
  CK(hipMalloc(&sink, (size_t)grid * kThreads * 4));
  CK(hipMemset(buf, 0x5A, kBytes + 4096));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct Shape {
    const char *name;
    double bytes;  // bytes of the buffer the launch reads or writes (each once)
  };
  auto run = [&](const char *name, double bytes, auto launch) {
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    printf("{\"kernel\": \"%s\", \"bytes\": %.0f, \"best_ms\": %.4f, \"gbs\": %.1f}\n", name, bytes, best,
           bytes / (best * 1e-3) / 1e9);
    fflush(stdout);
  };
  const size_t n16 = kBytes / 16, nch512 = kBytes / 512, nch32k = kBytes / 32768, n4 = kBytes / 4, nrec = kBytes / 64;
  run("stream16", (double)kBytes, [&] { stream16<<<grid, kThreads>>>((const uint4 *)buf, n16, sink); });
  run("u64_coal_ua", (double)(nch512 - 1) * 512, [&] { u64_coal_ua<<<grid, kThreads>>>(buf, nch512, sink); });
  run("u64_lane_ua", (double)(nch32k - 1) * 32768, [&] { u64_lane_ua<<<grid, kThreads>>>(buf, nch32k, sink); });
  run("u64_g4_ua", (double)(nch32k - 1) * 32768, [&] { u64_g4_ua<<<grid, kThreads>>>(buf, nch32k, sink); });
  run("b32_rows", (double)kBytes, [&] { b32_rows<<<grid, kThreads>>>((const uint32_t *)buf, n4, sink); });
  run("rec64_perm", (double)kBytes, [&] { rec64_perm<<<grid, kThreads>>>((const uint4 *)buf, nrec, sink); });
  // u16_perm reads 2 B of every 64-B record: the bytes of the lines it touches are the buffer
  run("u16_perm", (double)kBytes, [&] { u16_perm<<<grid, kThreads>>>((const uint16_t *)buf, nrec, sink); });
  run("wr_stream16", (double)kBytes, [&] { wr_stream16<<<grid, kThreads>>>((uint4 *)buf, n16); });
  run("wr_u64", (double)kBytes, [&] { wr_u64<<<grid, kThreads>>>((uint2 *)buf, kBytes / 8); });
  CK(hipDeviceSynchronize());
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
