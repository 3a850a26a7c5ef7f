// FETCH_SIZE calibration for the sparse kernel's wishlist access pattern
// (dev tool, run under rocprofv3 --pmc FETCH_SIZE on the GPU box).
//
// The guide's gfx950 rule (FETCH_SIZE = 1/2 of the bytes of a wide
// coalesced 16 B/lane stream) is calibrated only for that width.  The block
// build reads 200-byte wishlist rows of random children, 8 lanes per row,
// each lane 4 x 8-byte chunks.  This kernel repeats exactly that pattern over
// R distinct random rows of a 1M x 200 B table (no row read twice) and
// prints the number of distinct 128-byte lines it touches; FETCH_SIZE (x1024)
// of the `gather_rows` dispatch divided by lines x 128 is the correction
// factor for this pattern.  A second kernel streams the table with 16 B per
// lane (the guide's calibrated case) as a control.  A third (round 3e)
// repeats the tile build's packed-wishlist pattern: one lane per random
// 128-byte aligned row of a 1M x 128 B table, 8 x 16-byte loads (one line).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int ROW = 200;

__global__ void gather_rows(const uint8_t *tab, const int32_t *rows, int R, uint64_t *sink) {
  const int lane = threadIdx.x & 63;
  const int q = lane & 7;  // lane within the row group
  const int r = (blockIdx.x * blockDim.x + threadIdx.x) >> 3;
  uint64_t acc = 0;
  if (r < R) {
    const uint8_t *p = tab + (size_t)rows[r] * ROW;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int o = (c * 8 + q) * 8;  // chunk (c*8+q) of 25
      if (o < ROW) acc += *(const uint64_t *)(p + o);
    }
  }
  if (acc == 0x0123456789ABCDEFull) sink[0] = acc;  // keep the loads
}

__global__ void gather_lines(const uint4 *tab, const int32_t *rows, int R, uint64_t *sink) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t acc = 0;
  if (r < R) {
    const uint4 *p = tab + (size_t)rows[r] * 8;
#pragma unroll
    for (int c = 0; c < 8; ++c) {  // (64-bit terms: a 32-bit sum could never reach the sink test)
      const uint4 v = p[c];
      acc = acc * 31u + ((((uint64_t)v.x << 32) | v.y) ^ (((uint64_t)v.z << 32) | v.w));
    }
  }
  if (acc == 0x0123456789ABCDEFull) sink[0] = acc;  // keep the loads
}

__global__ void stream16(const uint4 *tab, size_t n16, uint64_t *sink) {
  uint64_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = tab[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x0123456789ABCDEFull) sink[0] = acc;
}

int main() {
  const int NC = 1000000, R = 954880;
  std::vector<int32_t> perm(NC);
  for (int i = 0; i < NC; ++i) perm[i] = i;
  uint64_t s = 2017;
  for (int i = NC - 1; i > 0; --i) {  // Fisher-Yates, splitmix-style LCG
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    const int j = (int)((s >> 33) % (uint64_t)(i + 1));
    std::swap(perm[i], perm[j]);
  }
  perm.resize(R);
  std::vector<uint8_t> seen((size_t)NC * ROW / 128 + 2, 0);
  size_t lines = 0;
  for (int r = 0; r < R; ++r) {
    const size_t b0 = (size_t)perm[r] * ROW, b1 = b0 + ROW - 1;
    for (size_t l = b0 / 128; l <= b1 / 128; ++l)
      if (!seen[l]) { seen[l] = 1; ++lines; }
  }
  uint8_t *tab;
  int32_t *rows;
  uint64_t *sink;
  CK(hipMalloc(&tab, (size_t)NC * ROW));
  CK(hipMalloc(&rows, (size_t)R * 4));
  CK(hipMalloc(&sink, 8));
  CK(hipMemset(tab, 1, (size_t)NC * ROW));
  CK(hipMemcpy(rows, perm.data(), (size_t)R * 4, hipMemcpyHostToDevice));
  const int threads = 256, blocks = (R * 8 + threads - 1) / threads;
  // flush the table out of the caches between runs by streaming another buffer
  uint8_t *flush;
  const size_t FL = (size_t)512 << 20;
  CK(hipMalloc(&flush, FL));
  CK(hipMemset(flush, 2, FL));
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(gather_rows, dim3(blocks), dim3(threads), 0, 0, tab, rows, R, sink);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(stream16, dim3(4096), dim3(256), 0, 0, (const uint4 *)flush, FL / 16, sink);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(stream16, dim3(4096), dim3(256), 0, 0, (const uint4 *)tab, (size_t)NC * ROW / 16, sink);
  CK(hipDeviceSynchronize());
  // packed-row gather: R distinct random 128-byte lines, one lane each
  uint4 *tab128;
  CK(hipMalloc(&tab128, (size_t)NC * 128));
  CK(hipMemset(tab128, 3, (size_t)NC * 128));
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(stream16, dim3(4096), dim3(256), 0, 0, (const uint4 *)flush, FL / 16, sink);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(gather_lines, dim3((R + threads - 1) / threads), dim3(threads), 0, 0, tab128, rows, R, sink);
  CK(hipDeviceSynchronize());
  printf("{\"rows\": %d, \"row_bytes\": %d, \"distinct_lines_128\": %zu, \"line_bytes\": %zu, "
         "\"useful_bytes\": %zu, \"stream16_bytes\": %zu, \"flush_bytes\": %zu, \"packed_line_bytes\": %zu}\n",
         R, ROW, lines, lines * 128, (size_t)R * ROW, (size_t)NC * ROW, FL, (size_t)R * 128);
  CK(hipFree(tab128));
  CK(hipFree(flush));
  CK(hipFree(tab));
  CK(hipFree(rows));
  CK(hipFree(sink));
  return 0;
}
