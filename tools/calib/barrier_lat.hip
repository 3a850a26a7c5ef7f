// Cross-wave step-exchange latency of the multi-wave block kernels (dev
// tool): one workgroup of NW waves alone on a CU, shader-clock ticks from
// s_memtime, per iteration of
//   0: s_barrier alone
//   1: lane 0 of every wave ds_min_u64 to one word, barrier, broadcast read
//      + readfirstlane (sap_solve_mw's step exchange, rotating 3 words)
//   2: the same with the wave DPP min of the high word in front (the whole
//      step argmin of the 4-wave kernel, without the relaxation)
//   3: every wave writes its own slot, barrier, reads all NW slots (b128)
//   4: as 3 with all 64 lanes writing the wave's uniform value
//   5: the full slot exchange of a 64-bit key (DPP min of the high words,
//      readlane of the unique holder's low word, all-lane write, read, min)
//   hipcc -O3 --offload-arch=gfx950 -o barrier_lat barrier_lat.hip && ./barrier_lat
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int ITER = 256;

__device__ __forceinline__ uint64_t tick() {
  asm volatile("s_waitcnt lgkmcnt(0) vmcnt(0)" ::: "memory");
  return __builtin_amdgcn_s_memtime();
}

template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t dmin(uint32_t x) {
  const uint32_t y = (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, CTRL, ROWMASK, 0xF, false);
  return y < x ? y : x;
}

__device__ __forceinline__ uint32_t wave_min(uint32_t x) {
  x = dmin<0xB1, 0xF>(x);
  x = dmin<0x4E, 0xF>(x);
  x = dmin<0x141, 0xF>(x);
  x = dmin<0x140, 0xF>(x);
  x = dmin<0x142, 0xA>(x);
  x = dmin<0x143, 0xC>(x);
  return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

template <int NW>
__global__ __launch_bounds__(NW * 64) void xlat(uint64_t *out, uint32_t seed) {
  __shared__ uint64_t red[8];
  __shared__ uint64_t slot[2][NW];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid < 8) red[tid] = ~0ull;
  __syncthreads();
  uint64_t acc = seed;
  uint64_t t0, t1;
  int k = 0;
#define TEST(body)                                                   \
  __syncthreads();                                                   \
  t0 = tick();                                                       \
  for (int it = 0; it < ITER; ++it) { body; }                        \
  t1 = tick();                                                       \
  if (tid == 0) out[blockIdx.x * 16 + k] = t1 - t0;                  \
  ++k;
  // 0: barrier alone
  TEST(__syncthreads());
  // 1: ds_min by lane 0 of each wave + barrier + broadcast read (rotating words)
  int par = 0;
  TEST({
    if (tid == 0) red[par == 2 ? 0 : par + 1] = ~0ull;
    if (lane == 0) __hip_atomic_fetch_min(red + par, acc + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __syncthreads();
    const uint64_t g = red[par];
    acc += (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)g) & 1u;
    par = par == 2 ? 0 : par + 1;
  });
  // 2: DPP wave min of a per-lane word in front of 1
  TEST({
    if (tid == 0) red[par == 2 ? 0 : par + 1] = ~0ull;
    const uint32_t x = (uint32_t)(acc * 2654435761u) ^ (uint32_t)tid;
    const uint32_t m = wave_min(x);
    if (x == m) __hip_atomic_fetch_min(red + par, ((uint64_t)m << 32) | (uint32_t)tid, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
    __syncthreads();
    const uint64_t g = red[par];
    acc += (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)g) & 1u;
    par = par == 2 ? 0 : par + 1;
  });
  // 3: own slot write + barrier + read all slots (double-buffered)
  int sb = 0;
  TEST({
    if (lane == 0) slot[sb][w] = acc + w;
    __syncthreads();
    uint64_t g = slot[sb][0];
    for (int q = 1; q < NW; ++q) g = g < slot[sb][q] ? g : slot[sb][q];
    acc += (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)g) & 1u;
    sb ^= 1;
  });
  // 4: every lane of a wave writes the wave's (uniform) value to its slot
  TEST({
    const uint64_t v = acc + w;
    slot[sb][w] = v;
    __syncthreads();
    uint64_t g = slot[sb][0];
    for (int q = 1; q < NW; ++q) g = g < slot[sb][q] ? g : slot[sb][q];
    acc += (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)g) & 1u;
    sb ^= 1;
  });
  // 5: the full slot exchange of a 64-bit key: DPP min of the high words, the
  //    low word of the (usually unique) holder by readlane, all-lane slot
  //    write, barrier, read all slots, min
  TEST({
    const uint32_t hi = (uint32_t)(acc * 2654435761u) ^ (uint32_t)(tid * 40503u);
    const uint32_t lo = (uint32_t)tid;
    const uint32_t m = wave_min(hi);
    const uint64_t tie = __builtin_amdgcn_ballot_w64(hi == m);
    uint32_t ml;
    if (__builtin_popcountll(tie) == 1)
      ml = (uint32_t)__builtin_amdgcn_readlane((int)lo, (int)__builtin_ctzll(tie));
    else
      ml = wave_min(hi == m ? lo : ~0u);
    slot[sb][w] = ((uint64_t)m << 32) | ml;
    __syncthreads();
    uint64_t g = slot[sb][0];
    for (int q = 1; q < NW; ++q) g = g < slot[sb][q] ? g : slot[sb][q];
    acc += (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)g) & 1u;
    sb ^= 1;
  });
  if (tid == 0) out[blockIdx.x * 16 + 15] = acc;
}

template <int NW>
void run(uint64_t *d, int G) {
  const char *names[] = {"s_barrier", "ds_min_u64 + barrier + read (rotating)",
                         "DPP min + ds_min_u64 + barrier + read", "slot write + barrier + read NW slots",
                         "all-lane slot write + barrier + read NW slots",
                         "DPP min + readlane + all-lane slot write + barrier + read + min"};
  CK(hipMemset(d, 0, (size_t)G * 16 * 8));
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(xlat<NW>, dim3(G), dim3(NW * 64), 0, 0, d, 1u + rep);
  CK(hipDeviceSynchronize());
  uint64_t *h = (uint64_t *)malloc((size_t)G * 16 * 8);
  CK(hipMemcpy(h, d, (size_t)G * 16 * 8, hipMemcpyDeviceToHost));
  for (int k = 0; k < 6; ++k) {
    double s = 0;
    for (int b = 0; b < G; ++b) s += (double)h[(size_t)b * 16 + k];
    printf("{\"waves_per_block\": %d, \"blocks\": %d, \"test\": \"%s\", \"cycles_per_iter\": %.2f}\n", NW, G,
           names[k], s / G / ITER);
  }
  free(h);
}

int main() {
  uint64_t *d;
  CK(hipMalloc(&d, 1024 * 16 * 8));
  run<2>(d, 1);
  run<4>(d, 1);
  run<8>(d, 1);
  run<4>(d, 512);
  return 0;
}
