// sh_common.h — host+device helpers shared by the gfx950 kernels and the
// host-side generator.  The Python mirror of every function here lives in
// santa_hip/sampler.py and must stay bit-identical (tests check both).
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SH_HD __host__ __device__ __forceinline__
#else
#define SH_HD static inline
#endif

// splitmix64 finaliser (Steele/Lea/Flood), the counter PRNG of the build.
SH_HD uint64_t sh_splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

SH_HD uint64_t sh_mix2(uint64_t a, uint64_t b) { return sh_splitmix64(a ^ sh_splitmix64(b)); }

// Feistel permutation of [0, count): replaces np.random.permutation(range(..))
// of mpi_single.py:123-124 with a keyed bijection evaluated per index.
struct ShFeistel {
  uint64_t key[4];
  uint32_t half;   // bits per half
  uint64_t mask;   // (1 << half) - 1
  uint64_t count;
};

SH_HD ShFeistel sh_feistel_make(uint64_t seed, uint64_t round, uint64_t count) {
  ShFeistel f;
  uint32_t bits = 2;
  while ((1ull << bits) < count) ++bits;
  if (bits & 1) ++bits;
  f.half = bits / 2;
  f.mask = (1ull << f.half) - 1ull;
  f.count = count;
  uint64_t base = sh_mix2(seed, round ^ 0x5851F42D4C957F2Dull);
  for (int r = 0; r < 4; ++r) f.key[r] = sh_splitmix64(base + (uint64_t)r);
  return f;
}

SH_HD uint64_t sh_feistel_encrypt(const ShFeistel &f, uint64_t x) {
  uint64_t L = x >> f.half, R = x & f.mask;
  for (int r = 0; r < 4; ++r) {
    uint64_t t = L ^ (sh_splitmix64(R ^ f.key[r]) & f.mask);
    L = R;
    R = t;
  }
  return (L << f.half) | R;
}

// Cycle-walking restriction of the 2^(2*half) bijection to [0, count).
SH_HD uint64_t sh_feistel_perm(const ShFeistel &f, uint64_t x) {
  uint64_t y = sh_feistel_encrypt(f, x);
  while (y >= f.count) y = sh_feistel_encrypt(f, y);
  return y;
}

// Device-generated LSAP cost for the pure-solver sweep (BASELINE config 5).
SH_HD uint64_t sh_hash_cost(uint64_t seed, uint64_t b, uint64_t i, uint64_t j) {
  uint64_t x = (b << 40) ^ (i << 20) ^ j;
  return sh_splitmix64(seed ^ sh_splitmix64(x));
}
