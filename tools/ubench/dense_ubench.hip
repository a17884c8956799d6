// Micro-benchmark (diagnostic, not shipped): cycles per 128 x 128 dense layer of the resident
// kernel's network chain (search_res_kernel: activations in padded LDS rows, one barrier per layer,
// weights in registers) for the 256-thread layout (one wave per SIMD, lane = 4 columns over a K
// eighth, reduce_d4) against a 512-thread layout (two waves per SIMD, lane = 2 columns over a K
// eighth, 32 FMAs per lane): does the second wave per SIMD hide the first's LDS / DPP / barrier
// latency? One workgroup per CU (256 workgroups), NL layers per "simulation", S simulations.
// Build: hipcc -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 -o dense_ubench dense_ubench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr int kRow = 132;  // padded activation row (lzm_search_res.h kRRow)
constexpr int S = 50, NL = 6;

template <int C>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), C, 0xF, 0xF, false));
}
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void fma4(float4 v, float4 q, float *a) {
  f2 lo = {a[0], a[1]}, hi = {a[2], a[3]};
  lo = __builtin_elementwise_fma((f2){v.x, v.y}, (f2){q.x, q.y}, lo);
  hi = __builtin_elementwise_fma((f2){v.z, v.w}, (f2){q.z, q.w}, hi);
  a[0] = lo.x; a[1] = lo.y; a[2] = hi.x; a[3] = hi.y;
}
__device__ __forceinline__ int rpad(int c) { return c + ((c >> 6) << 2); }

// 256 threads: lane owns columns 4 (l >> 3) + c over K eighth 16 (l & 7)
__device__ __forceinline__ float layer256(const float *x, const float4 *w) {
  const int e = threadIdx.x & 7;
  const float4 *x4 = reinterpret_cast<const float4 *>(x) + 4 * e + (e >> 2);
  float4 xv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) xv[j] = x4[j];
  float a[4][4] = {};
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int c = 0; c < 4; ++c) fma4(xv[j], w[4 * j + c], a[c]);
  float h[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) h[c] = (a[c][0] + a[c][1]) + (a[c][2] + a[c][3]);
  const bool lo = e < 4;
  float k0 = lo ? h[0] : h[2], k1 = lo ? h[1] : h[3];
  k0 += dpp<0x141>(lo ? h[2] : h[0]);
  k1 += dpp<0x141>(lo ? h[3] : h[1]);
  const bool q = (e & 2) == 0;
  float m = q ? k0 : k1;
  m += dpp<0x4E>(q ? k1 : k0);
  return m + dpp<0xB1>(m);
}
// 512 threads: lane owns columns 2 (l >> 3) + c over K eighth 16 (l & 7)
__device__ __forceinline__ float layer512(const float *x, const float4 *w) {
  const int e = threadIdx.x & 7;
  const float4 *x4 = reinterpret_cast<const float4 *>(x) + 4 * e + (e >> 2);
  float4 xv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) xv[j] = x4[j];
  float a[2][4] = {};
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int c = 0; c < 2; ++c) fma4(xv[j], w[2 * j + c], a[c]);
  const float h0 = (a[0][0] + a[0][1]) + (a[0][2] + a[0][3]), h1 = (a[1][0] + a[1][1]) + (a[1][2] + a[1][3]);
  const bool lo = e < 4;
  float u = lo ? h0 : h1;
  u += dpp<0x141>(lo ? h1 : h0);
  u += dpp<0x4E>(u);
  return u + dpp<0xB1>(u);
}

// WL: the two layers' weights in LDS ([slot][lane] float4, as the kernel's fc_dynamics[1] /
// fc_dynamics_2[0]) instead of registers
template <int T, bool WL = false>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(T / 256, T / 256))) void chain_kernel(
    const float4 *gw, unsigned long long *cyc, float *out) {
  constexpr int NW = T == 256 ? 16 : 8;  // float4 weights per lane per layer
  __shared__ float act[2][kRow];
  extern __shared__ float4 lw[];  // WL: [2][NW][T]
  float4 w[2][WL ? 1 : NW];  // two register layers, used alternately
#pragma unroll
  for (int l = 0; l < 2; ++l)
#pragma unroll
    for (int j = 0; j < NW; ++j) {
      if (WL) lw[(l * NW + j) * T + threadIdx.x] = gw[(l * NW + j) * T + threadIdx.x];
      else w[l][j] = gw[(l * NW + j) * T + threadIdx.x];
    }
  if (threadIdx.x < kRow) act[0][threadIdx.x] = 0.01f * (threadIdx.x % 7);
  __syncthreads();
  const int tid = threadIdx.x;
  const int col = T == 256 ? 4 * (tid >> 3) + ((tid & 7) >> 1) : 2 * (tid >> 3) + ((tid & 7) >> 2);
  const bool writer = T == 256 ? (tid & 1) == 0 : (tid & 3) == 0;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  int cur = 0;
  for (int s = 0; s < S; ++s) {
#pragma unroll
    for (int l = 0; l < NL; ++l) {
      float z;
      if (WL) {
        float4 wl[NW];
#pragma unroll
        for (int j = 0; j < NW; ++j) wl[j] = lw[((l & 1) * NW + j) * T + tid];
        z = T == 256 ? layer256(act[cur], wl) : layer512(act[cur], wl);
      } else {
        z = T == 256 ? layer256(act[cur], w[l & 1]) : layer512(act[cur], w[l & 1]);
      }
      if (writer) act[cur ^ 1][rpad(col)] = fmaxf(z, 0.0f) * 0.5f + 0.001f;
      __syncthreads();
      cur ^= 1;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
  if (tid < 128) out[blockIdx.x * 128 + tid] = act[cur][rpad(tid)];
}

template <int T, bool WL = false>
static double run(const float4 *w, unsigned long long *cyc, float *out, int G) {
  const size_t lds = WL ? 2 * (T == 256 ? 16 : 8) * T * sizeof(float4) : 0;
  if (WL) hipFuncSetAttribute((const void *)chain_kernel<T, WL>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  chain_kernel<T, WL><<<G, T, lds>>>(w, cyc, out);
  hipDeviceSynchronize();
  std::vector<unsigned long long> h(G);
  double best = 1e30;
  for (int r = 0; r < 5; ++r) {
    chain_kernel<T, WL><<<G, T, lds>>>(w, cyc, out);
    hipDeviceSynchronize();
    hipMemcpy(h.data(), cyc, G * 8, hipMemcpyDeviceToHost);
    double m = 0;
    for (int g = 0; g < G; ++g) m += (double)h[g];
    m /= G;
    if (m < best) best = m;
  }
  return best / (S * NL);  // s_memtime ticks per layer
}

int main() {
  const int G = 256;
  float4 *w;
  unsigned long long *cyc;
  float *out;
  hipMalloc(&w, 2 * 16 * 512 * sizeof(float4));
  hipMalloc(&cyc, G * 8);
  hipMalloc(&out, G * 128 * 4);
  std::vector<float> hw(2 * 16 * 512 * 4);
  for (size_t i = 0; i < hw.size(); ++i) hw[i] = 0.01f * (float)((i * 2654435761u) % 200) / 200.0f - 0.005f;
  hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice);
  const double c256 = run<256>(w, cyc, out, G);
  const double c512 = run<512>(w, cyc, out, G);
  const double l256 = run<256, true>(w, cyc, out, G);
  const double l512 = run<512, true>(w, cyc, out, G);
  printf("{\"ticks_per_layer_256\": %.1f, \"ticks_per_layer_512\": %.1f, \"ratio\": %.3f, \"lds_weights_256\": %.1f, "
         "\"lds_weights_512\": %.1f, \"note\": \"s_memtime ticks, %d layers x %d sims, %d workgroups\"}\n",
         c256, c512, c512 / c256, l256, l512, NL, S, G);
  return 0;
}
