// Micro-benchmark (diagnostic, not shipped): cycles per level of the resident kernel's selection
// walk (descend_small<2>, lzm_search_res.h) in isolation, on a synthetic full binary tree in LDS
// (depth D, walk ends at a two-way tie among unexpanded children like most real simulations),
// with NP float4 per lane held live across the walk to emulate the resident kernel's register
// pressure (its network weights stay in registers for the whole launch).
// Build: hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 -o walk_ubench walk_ubench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../lightzero_amd/csrc/lzm_search_res.h"
using namespace lzm;

constexpr int D = 6, NLAT = (1 << D) - 1, CAP = 1 + 2 * (NLAT + 1), REPS = 200;

template <int NP, int V>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void walk_kernel(
    const float4 *gcs, const float2 *gnq, unsigned long long *cyc, int *out, const float4 *pin, const float4 *gmm,
    const int *gi) {
  float4 hold[NP > 0 ? NP : 1];
#pragma unroll
  for (int j = 0; j < NP; ++j) hold[j] = pin[j * 256 + threadIdx.x];
  __shared__ float4 cs[CAP];
  __shared__ float2 nq[NLAT + 1];
  __shared__ int path[64], pact[64], lg[4];
  __shared__ NodeMeta meta[1];
  __shared__ int dec[NLAT + 1];
  __shared__ float2 chain[64];
  for (int e = threadIdx.x; e < CAP; e += 256) cs[e] = gcs[e];
  for (int e = threadIdx.x; e <= NLAT; e += 256) nq[e] = gnq[e];
  __syncthreads();
  for (int e = threadIdx.x; e <= NLAT; e += 256) dec[e] = a2_decision(cs[1 + 2 * e], cs[2 + 2 * e], 2);
  if (threadIdx.x < 2) lg[threadIdx.x] = threadIdx.x;
  if (threadIdx.x == 0) {
    lg[2] = 2;
    meta[0].latent = 0;
  }
  __syncthreads();
  TreeView t;
  t.A = gi[0]; t.cap = CAP; t.B = 1; t.depth_cap = gi[1]; t.path = path; t.path_act = pact; t.legal = lg; t.nlegal = lg + 2;
  t.meta = meta;
  int acc = 0;
  if (threadIdx.x < 64) {
    const float4 mm = gmm[0];  // run-time values, as in the search kernel
    int rleg[2] = {gi[2], gi[3]};
    const int nleg = gi[4], players = gi[5], vtp = gi[6];
    auto nodraw = [](int) -> uint32_t { return 0u; };
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < REPS; ++r) {
      TieInfo ti;
      if (V == 2) {
        // floor: a bare pointer chase down child 0 (one dependent LDS read per level)
        int lat = 0, len = 0;
        while (lat >= 0 && len < t.depth_cap) {
          lat = __float_as_int(cs[1 + 2 * lat].z);
          ++len;
        }
        acc += len + 1;
      } else {
        Descent d = V == 0 ? descend_small<2, true>(t, nq, cs, mm, vtp, players, rleg, nleg, nodraw, &ti)
                  : V == 1 ? descend_a2<true, decltype(nodraw), 0>(t, nq, dec, cs, mm, vtp, players, rleg, nleg, nodraw, &ti)
                  : V == 3 ? descend_a2f<true>(t, nq, dec, cs, mm, vtp, players, rleg, nleg, nodraw, &ti)
                  : V == 4 ? descend_a2<true, decltype(nodraw), 4>(t, nq, dec, cs, mm, vtp, players, rleg, nleg, nodraw, &ti,
                                                                   nullptr, nullptr, chain)
                           : descend_a2<true, decltype(nodraw), 5>(t, nq, dec, cs, mm, vtp, players, rleg, nleg, nodraw, &ti,
                                                                   nullptr, nullptr, chain);
        acc += d.len + ti.status;
      }
      __builtin_amdgcn_s_waitcnt(0);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
      cyc[blockIdx.x] = t1 - t0;
      out[blockIdx.x] = acc;
    }
  }
  float sacc = 0.0f;
#pragma unroll
  for (int j = 0; j < NP; ++j) sacc += hold[j].x * hold[j].y + hold[j].z * hold[j].w;
  if (sacc == 12345.0f) out[0] = 7;
}

template <int NP, int V>
void run(const float4 *dcs, const float2 *dnq, unsigned long long *dc, int *dout, const float4 *dpin, int G,
         const float4 *dmm, const int *dgi) {
  for (int it = 0; it < 3; ++it)
    hipLaunchKernelGGL((walk_kernel<NP, V>), dim3(G), dim3(256), 0, 0, dcs, dnq, dc, dout, dpin, dmm, dgi);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> c(G);
  std::vector<int> o(G);
  (void)hipMemcpy(c.data(), dc, 8 * G, hipMemcpyDeviceToHost);
  (void)hipMemcpy(o.data(), dout, 4 * G, hipMemcpyDeviceToHost);
  double s = 0;
  for (auto v : c) s += (double)v;
  const double per_walk = s / G / REPS;
  const double lvl = (double)o[0] / REPS - 1;  // len + status(1)
  printf("variant %d pinned %3d floats/lane: %.0f cycles per walk, mean len %.2f, %.0f cycles per level\n", V, NP * 4, per_walk, lvl,
         per_walk / lvl);
}

static float i2f(int v) {
  float f;
  memcpy(&f, &v, 4);
  return f;
}

int main() {
  std::vector<float4> cs(CAP);
  std::vector<float2> nq(NLAT + 1);
  srand(1);
  auto rnd = []() { return (float)rand() / 2147483648.0f; };
  // latent L's children are nodes 1 + 2L + j; expanded children get BFS latents
  int next = 1;
  for (int L = 0; L < NLAT; ++L)
    for (int j = 0; j < 2; ++j) {
      const int c = 1 + 2 * L + j;
      const bool exp = next < NLAT;
      const int cl = exp ? next++ : -1;
      // expanded children: visited, distinct scores; leaves: unvisited, equal prior scores (tie)
      cs[c] = make_float4(exp ? rnd() : 0.0f, exp ? rnd() : 0.0f, i2f(cl), i2f(exp ? 1 : 0));
    }
  for (int L = 0; L <= NLAT; ++L) nq[L] = make_float2(rnd(), i2f(L < NLAT / 2 ? 2 : 0));
  float4 *dcs, *dpin;
  float2 *dnq;
  unsigned long long *dc;
  int *dout;
  const int G = 256;
  (void)hipMalloc(&dcs, sizeof(float4) * CAP);
  (void)hipMalloc(&dnq, sizeof(float2) * (NLAT + 1));
  (void)hipMalloc(&dc, 8 * G);
  (void)hipMalloc(&dout, 4 * G);
  (void)hipMalloc(&dpin, sizeof(float4) * 256 * 120);
  (void)hipMemset(dpin, 0, sizeof(float4) * 256 * 120);
  (void)hipMemcpy(dcs, cs.data(), sizeof(float4) * CAP, hipMemcpyHostToDevice);
  (void)hipMemcpy(dnq, nq.data(), sizeof(float2) * (NLAT + 1), hipMemcpyHostToDevice);
  const float4 hmm = make_float4(1.0f, 0.0f, 0.01f, 0.0f);
  const int hgi[8] = {2, 64, 0, 1, 2, 1, -1, 0};
  float4 *dmm;
  int *dgi;
  (void)hipMalloc(&dmm, sizeof(float4));
  (void)hipMalloc(&dgi, sizeof(hgi));
  (void)hipMemcpy(dmm, &hmm, sizeof(float4), hipMemcpyHostToDevice);
  (void)hipMemcpy(dgi, hgi, sizeof(hgi), hipMemcpyHostToDevice);
  run<0, 0>(dcs, dnq, dc, dout, dpin, G, dmm, dgi);
  run<0, 1>(dcs, dnq, dc, dout, dpin, G, dmm, dgi);
  run<0, 2>(dcs, dnq, dc, dout, dpin, G, dmm, dgi);
  run<0, 3>(dcs, dnq, dc, dout, dpin, G, dmm, dgi);

  return 0;
}
