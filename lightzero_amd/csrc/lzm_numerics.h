// lzm_numerics.h — bit-exact scalar numerics shared by the tree kernels (gfx950 device code).
//
// glibc_expf: the reference tree computes priors with the host libm expf
// (ctree_muzero/lib/cnode.cpp:129, float overload). On x86-64 glibc 2.35 dispatches to the
// FMA build of sysdeps/ieee754/flt-32/e_expf.c: a 32-entry 2^(k/32) table and a cubic in
// double precision. This is a restatement of that published algorithm with the same
// constants and the same fused multiply-adds; it equals host expf on every float in
// [-103.97, 0] (exhaustive check: tests/test_numerics.py, scripts under tests/).
//
// glibc rand(): srandom_r/random_r TYPE_3 (additive lagged Fibonacci, lags 31/3), used by
// cselect_child (cnode.cpp:592) after srand(tv_usec) (common_lib/utils.cpp:25).
//
// philox4x32_10: counter-based stream for the LZM_RNG_FAST mode (Salmon et al., SC'11).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lzm {

__device__ __constant__ static const uint64_t kExp2fTab[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};

// tab: the 2^(k/32) table (kExp2fTab, or a copy of it in LDS: a kernel that keeps global loads
// in flight across the call then waits only for this LDS read, not for every outstanding load).
__device__ inline float glibc_expf(float x, const uint64_t *tab = kExp2fTab) {
  const double kInvLn2N = 0x1.71547652b82fep+5;  // 32/ln2
  const double kShift = 0x1.8p+52;
  const double C0 = 0x1.c6af84b912394p-20, C1 = 0x1.ebfce50fac4f3p-13, C2 = 0x1.62e42ff0c52d6p-6;
  uint32_t ux = __float_as_uint(x);
  uint32_t abstop = (ux >> 20) & 0x7ff;
  if (abstop >= 0x42b) {  // |x| >= 88 or x is nan
    if (ux == 0xff800000u) return 0.0f;
    if (abstop >= 0x7f8) return x + x;
    if (x > 0x1.62e42ep6f) return __uint_as_float(0x7f800000u);  // overflow
    if (x < -0x1.9fe368p6f) return 0.0f;                        // underflow
  }
  double xd = (double)x;
  double kd = __fma_rn(kInvLn2N, xd, kShift);
  uint64_t ki = (uint64_t)__double_as_longlong(kd);
  kd -= kShift;
  double r = __fma_rn(kInvLn2N, xd, -kd);
  uint64_t t = tab[ki % 32];
  t += ki << 47;
  double s = __longlong_as_double((long long)t);
  double z = __fma_rn(C0, r, C1);
  double r2 = r * r;
  double y = __fma_rn(C2, r, 1.0);
  y = __fma_rn(z, r2, y);
  y = y * s;
  return (float)y;
}

// glibc srandom_r initial state (31 words) for `seed` (0 -> 1), Schrage's method.
__device__ inline void glibc_seed_state(uint32_t seed, uint32_t *z0) {
  if (seed == 0) seed = 1;
  int32_t word = (int32_t)seed;
  z0[0] = seed;
  for (int i = 1; i < 31; ++i) {
    long long hi = word / 127773;
    long long lo = word % 127773;
    long long w = 16807 * lo - 2836 * hi;
    if (w < 0) w += 2147483647;
    word = (int32_t)w;
    z0[i] = (uint32_t)word;
  }
}

__device__ inline uint4 philox4x32_10(uint4 ctr, uint2 key) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(M0, ctr.x), lo0 = M0 * ctr.x;
    uint32_t hi1 = __umulhi(M1, ctr.z), lo1 = M1 * ctr.z;
    ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
    key.x += W0;
    key.y += W1;
  }
  return ctr;
}

}  // namespace lzm
