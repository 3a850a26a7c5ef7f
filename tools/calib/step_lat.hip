// Instruction latency / issue-cost microbenchmarks for the Dijkstra step of
// the block kernels (dev tool; one wave alone on a SIMD, shader-clock ticks
// from s_memtime).  Each test runs a 32-instruction unrolled body 64 times;
// the printed figure is cycles per body-instruction (or per named unit).
//   hipcc -O3 --offload-arch=gfx950 -o step_lat step_lat.hip && ./step_lat
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

constexpr int ITER = 64;
#define R4(x) x x x x
#define R8(x) R4(x) R4(x)
#define R32(x) R4(R4(x)) R4(R4(x))

__device__ __forceinline__ uint64_t tick() {
  asm volatile("s_waitcnt lgkmcnt(0) vmcnt(0)" ::: "memory");
  return __builtin_amdgcn_s_memtime();
}

__global__ void lat(uint64_t *out, uint32_t seed) {
  __shared__ uint64_t lds[1024];
  const int lane = threadIdx.x;
  for (int i = lane; i < 1024; i += 64) lds[i] = (uint64_t)((i + 1) & 1023) * 8;
  __syncthreads();
  uint32_t a = seed + lane, b = seed * 3 + 1, c = lane * 7, d = lane ^ 5, e = 9, f = 11, g = 13, h = 17;
  uint64_t A = seed + lane, B = 3, C = 5, D = 7;
  int k = 0;
  uint64_t t0, t1;
#define TEST(body)                                \
  t0 = tick();                                    \
  for (int it = 0; it < ITER; ++it) { body; }     \
  t1 = tick();                                    \
  if (lane == 0) out[blockIdx.x * 64 + k] = t1 - t0; \
  ++k;
  // 0: dependent v_add_u32 chain
  TEST(asm volatile(R32("v_add_u32 %0, %0, %1\n\t") : "+v"(a) : "v"(b)));
  // 1: independent v_add_u32 (8 chains)
  TEST(asm volatile(R4("v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
                       "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8\n\t")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(lane)));
  // 2: dependent v_lshl_add_u64 chain
  TEST(asm volatile(R32("v_lshl_add_u64 %0, %0, 0, %1\n\t") : "+v"(A) : "v"(B)));
  // 3: independent v_lshl_add_u64 (4 chains)
  TEST(asm volatile(R8("v_lshl_add_u64 %0, %0, 0, %4\n\tv_lshl_add_u64 %1, %1, 0, %4\n\t"
                       "v_lshl_add_u64 %2, %2, 0, %4\n\tv_lshl_add_u64 %3, %3, 0, %4\n\t")
                   : "+v"(A), "+v"(B), "+v"(C), "+v"(D) : "v"(A)));
  // 4: dependent 64-bit running min: v_cmp_lt_u64 + 2 v_cndmask (cost per triple)
  TEST(asm volatile("v_mov_b32 v62, %0\n\tv_mov_b32 v63, 0\n\tv_mov_b32 v64, 3\n\tv_mov_b32 v65, 0\n\t"
                    R32("v_cmp_lt_u64 vcc, v[64:65], v[62:63]\n\tv_cndmask_b32 v62, v62, v64, vcc\n\t"
                        "v_cndmask_b32 v63, v63, v65, vcc\n\t")
                   :: "v"(a) : "vcc", "v62", "v63", "v64", "v65"));
  // 5: DPP 32-bit min reduction over the wave (6 levels + readlane), per reduction
  {
    uint32_t x = a, r = 0;
    TEST(asm volatile(R32(
        "s_nop 1\n\tv_min_u32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\tv_min_u32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\tv_min_u32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\tv_min_u32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\tv_min_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 1\n\tv_min_u32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
        "s_nop 1\n\tv_readlane_b32 %1, %0, 63\n\tv_add_u32 %0, %1, %0\n\t") : "+v"(x), "+s"(r)));
    a += x;
  }
  // 6: VALU -> SALU -> VALU round trip: v_readlane, s_add, v_add with the SGPR
  {
    uint32_t s = 1;
    TEST(asm volatile(R32("v_readlane_b32 %1, %0, 5\n\ts_add_u32 %1, %1, 1\n\tv_add_u32 %0, %1, %0\n\t")
                     : "+v"(a), "+s"(s) :: "scc"));
  }
  // 7: dependent ds_read_b64 chain (address = previous value)
  {
    uint32_t p = (lane & 7) * 8;
    TEST(asm volatile(R32("ds_read_b32 %0, %0\n\ts_waitcnt lgkmcnt(0)\n\t") : "+v"(p)));
    a += p;
  }
  // 8: ds_write_b64 then ds_read_b128 at the written row, dependent
  {
    uint32_t p = lane * 16;
    uint64_t v = 0;
    TEST(asm volatile(R32("ds_write_b64 %0, %1\n\tds_read_b128 v[60:63], %0\n\ts_waitcnt lgkmcnt(0)\n\tv_and_b32 %0, 0x3f0, v60\n\t")
                     : "+v"(p), "+v"(v) :: "v60", "v61", "v62", "v63", "memory"));
    a += p;
  }
  // 9: v_readfirstlane + s_cselect + s_and chain (SGPR decode), per triple
  {
    uint32_t s = 0;
    TEST(asm volatile(R32("v_readfirstlane_b32 %1, %0\n\ts_cmp_eq_u32 %1, 0\n\ts_cselect_b32 %1, %1, 7\n\tv_mov_b32 %0, %1\n\t")
                     : "+v"(a), "+s"(s) :: "scc"));
  }
  // 10: independent v_cmp_lt_i64 into separate SGPR pairs (issue)
  TEST(asm volatile(R4("v_cmp_lt_i64 s[40:41], %0, %1\n\tv_cmp_lt_i64 s[42:43], %1, %2\n\tv_cmp_lt_i64 s[44:45], %2, %3\n\tv_cmp_lt_i64 s[46:47], %3, %0\n\t"
                       "v_cmp_lt_i64 s[48:49], %0, %2\n\tv_cmp_lt_i64 s[50:51], %1, %3\n\tv_cmp_lt_i64 s[52:53], %2, %0\n\tv_cmp_lt_i64 s[54:55], %3, %1\n\t")
                   :: "v"(A), "v"(B), "v"(C), "v"(D) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47",
                      "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55"));
  // 11: independent v_cndmask_b32 with SGPR masks
  TEST(asm volatile(R4("v_cndmask_b32 %0, %0, %8, s[40:41]\n\tv_cndmask_b32 %1, %1, %8, s[42:43]\n\tv_cndmask_b32 %2, %2, %8, s[44:45]\n\tv_cndmask_b32 %3, %3, %8, s[46:47]\n\t"
                       "v_cndmask_b32 %4, %4, %8, s[40:41]\n\tv_cndmask_b32 %5, %5, %8, s[42:43]\n\tv_cndmask_b32 %6, %6, %8, s[44:45]\n\tv_cndmask_b32 %7, %7, %8, s[46:47]\n\t")
                   : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h) : "v"(lane)));
  // 12: independent SALU (8 chains of s_add_u32)
  {
    uint32_t s0 = 1, s1 = 2, s2 = 3, s3 = 4;
    TEST(asm volatile(R4("s_add_u32 %0, %0, 3\n\ts_add_u32 %1, %1, 3\n\ts_add_u32 %2, %2, 3\n\ts_add_u32 %3, %3, 3\n\t"
                         "s_add_u32 %0, %0, 5\n\ts_add_u32 %1, %1, 5\n\ts_add_u32 %2, %2, 5\n\ts_add_u32 %3, %3, 5\n\t")
                     : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3) :: "scc"));
    a += s0 + s1 + s2 + s3;
  }
  // 13: v_min3_u32 dependent chain
  TEST(asm volatile(R32("v_min3_u32 %0, %0, %1, %2\n\t") : "+v"(a) : "v"(b), "v"(c)));
  // 14: v_readlane_b32 independent (8 into different SGPRs)
  TEST(asm volatile(R4("v_readlane_b32 s40, %0, 1\n\tv_readlane_b32 s41, %0, 2\n\tv_readlane_b32 s42, %0, 3\n\tv_readlane_b32 s43, %0, 4\n\t"
                       "v_readlane_b32 s44, %0, 5\n\tv_readlane_b32 s45, %0, 6\n\tv_readlane_b32 s46, %0, 7\n\tv_readlane_b32 s47, %0, 8\n\t")
                   :: "v"(a) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47"));
  // 15: ds_read_b128 independent issue (8 per body / 4 repeats)
  {
    uint32_t p = lane * 16;
    uint32_t q[4];
    TEST(asm volatile(R32("ds_read_b128 v[60:63], %0\n\t") "s_waitcnt lgkmcnt(0)\n\t" :: "v"(p) : "v60", "v61", "v62", "v63", "memory"));
    (void)q;
  }
  // 16: permlane32_swap (gfx950) dependent
  TEST(asm volatile(R32("v_permlane32_swap_b32 %0, %1\n\t") : "+v"(a), "+v"(b)));
  // 17: v_cmp + v_cndmask pair dependent (32-bit running min)
  TEST(asm volatile(R32("v_cmp_lt_u32 vcc, %1, %0\n\tv_cndmask_b32 %0, %0, %1, vcc\n\t") : "+v"(a) : "v"(c) : "vcc"));
  // 18: 64-lane ds_min_u64 to one LDS word, then broadcast ds_read_b64 and re-arm
  //     (per group: write ~0, min, read, wait, use)
  {
    uint32_t p = 4096;  // one word, same address for every lane
    uint64_t key = ((uint64_t)(lane * 2654435761u) << 20) | lane, got = 0;
    TEST(asm volatile(R32("ds_write_b64 %0, %3\n\tds_min_u64 %0, %1\n\tds_read_b64 %2, %0\n\ts_waitcnt lgkmcnt(0)\n\t"
                          "v_lshl_add_u64 %1, %1, 0, %2\n\t")
                     : "+v"(p), "+v"(key), "=v"(got) : "v"(~0ull) : "memory"));
    a += (uint32_t)got;
  }
  // 19: 64-lane ds_min_u32 + read (32-bit form)
  {
    uint32_t p = 4096;
    uint32_t key = lane * 2654435761u, got = 0;
    TEST(asm volatile(R32("ds_write_b32 %0, %3\n\tds_min_u32 %0, %1\n\tds_read_b32 %2, %0\n\ts_waitcnt lgkmcnt(0)\n\t"
                          "v_add_u32 %1, %1, %2\n\t")
                     : "+v"(p), "+v"(key), "=v"(got) : "v"(~0u) : "memory"));
    a += got;
  }
  // 20: s_nop 1 alone (per nop)
  TEST(asm volatile(R32("s_nop 1\n\t")));
  // 21: v_mov_b32_dpp row_shr:1 dependent with s_nop 1 (per pair)
  TEST(asm volatile(R32("s_nop 1\n\tv_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n\t") : "+v"(a)));
  if (lane == 0) out[blockIdx.x * 64 + 63] = a + b + c + d + e + f + g + h + (uint32_t)(A + B + C + D);
}

int main() {
  const char *names[] = {"v_add_u32 dep", "v_add_u32 indep", "v_lshl_add_u64 dep", "v_lshl_add_u64 indep",
                         "cmp_u64+2cndmask dep (per triple)", "DPP min reduction + readlane (per reduction)",
                         "readlane->s_add->v_add (per triple)", "ds_read_b32 dep + wait (per read)",
                         "ds_write_b64+ds_read_b128+wait+v_and (per group)",
                         "readfirstlane->s_cmp->s_cselect->v_mov (per group)", "v_cmp_lt_i64 indep",
                         "v_cndmask indep", "s_add indep", "v_min3 dep", "v_readlane indep",
                         "ds_read_b128 indep (issue)", "v_permlane32_swap dep", "v_cmp_u32+cndmask dep (per pair)",
                         "64-lane ds_min_u64 + read + wait (per group)", "64-lane ds_min_u32 + read + wait (per group)",
                         "s_nop 1", "s_nop 1 + dpp mov dep (per pair)"};
  const int grids[] = {1, 1024, 2048, 4096};
  uint64_t *d;
  CK(hipMalloc(&d, 4096 * 64 * 8));
  for (int gi = 0; gi < 4; ++gi) {
    const int G = grids[gi];
    CK(hipMemset(d, 0, (size_t)G * 64 * 8));
    for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(lat, dim3(G), dim3(64), 0, 0, d, 1u + rep);
    CK(hipDeviceSynchronize());
    uint64_t *h = (uint64_t *)malloc((size_t)G * 64 * 8);
    CK(hipMemcpy(h, d, (size_t)G * 64 * 8, hipMemcpyDeviceToHost));
    for (int k = 0; k < 22; ++k) {
      double s = 0;
      for (int b = 0; b < G; ++b) s += (double)h[(size_t)b * 64 + k];
      printf("{\"waves\": %d, \"test\": \"%s\", \"cycles_per_unit\": %.2f}\n", G, names[k], s / G / (ITER * 32.0));
    }
    free(h);
  }
  return 0;
}
