// lzm_initial.h — MuZeroModelMLP.initial_inference in one launch (the collect step's first op).
//
// MuZeroPolicy._forward_collect (muzero.py:617-690) runs the model's initial_inference on the
// observations before every search: representation (muzero_model_mlp.py:145-177,
// common.py:467-517: Linear O->H, BatchNorm, GELU(tanh), Linear H->H, SimNorm over groups of 8)
// then prediction (common.py:883-971: two Linear+BN+ReLU, value head Linear+BN+ReLU -> Linear to
// the support, policy head Linear+BN+ReLU -> Linear to A). As PyTorch modules that is ~20 launches
// (GEMMs, eval BatchNorm, activations, softmax) of a few microseconds each around tiny matrices; at
// the bench shape it was ~1/8 of the whole collect step. Here one workgroup takes kIiEnvs envs (1:
// 256 workgroups at B = 256, 18.6 us; 4 envs per workgroup: 24 us),
// keeps their activations in LDS and runs every layer (BatchNorm folded on the host in float64):
// a layer of N outputs over K inputs maps thread t to column t % N and K slice t / N (N < 256) or
// to columns t, t + 256, ... (N >= 256); K slices are summed in slice order (deterministic).
// Weights: per layer W[K][N] (torch weight transposed) + bias[N], read straight from L2 with the
// k loop unrolled so a batch of loads is in flight.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lzm {

constexpr int kIiThreads = 256;
constexpr int kIiEnvs = 1;
constexpr int kIiMaxW = 1024;  // widest activation row kept in LDS (support <= 1024)
constexpr int kIiLayers = 9;   // R1 R2 | P1 P2 | V1 V2 | Q1 Q2 (+ spare)

struct IiArgs {
  int B, O, H, F, V, A, group;
  const float *obs;                       // [B][O]
  const float *w[kIiLayers], *b[kIiLayers];  // 0 R1 (O->H, GELU), 1 R2 (H->H), 2 P1, 3 P2 (H->H, ReLU),
                                          // 4 V1 (H->F, ReLU), 5 V2 (F->V), 6 Q1 (H->F, ReLU), 7 Q2 (F->A)
  float *latent, *value, *policy;         // [B][H], [B][V], [B][A]
};

__device__ inline float ii_act(float v, int act) {
  if (act == 1) return fmaxf(v, 0.0f);
  if (act == 2) {
    // GELU, tanh approximation (torch: 0.5 x (1 + tanh(sqrt(2/pi) (x + 0.044715 x^3))))
    const float kBeta = 0.7978845608028654f, kKappa = 0.044715f;
    const float inner = kBeta * (v + kKappa * v * v * v);
    return 0.5f * v * (1.0f + tanhf(inner));
  }
  return v;
}

// out[e][n] = act(sum_k in[e][k] W[k][n] + b[n]) for the workgroup's envs; in / out / part in LDS
__device__ inline void ii_dense(const float *__restrict__ W, const float *__restrict__ bias, int K, int N,
                                const float *in, int ldi, float *out, int ldo, int act, float *part) {
  const int t = threadIdx.x;
  if (N >= kIiThreads) {
    for (int n = t; n < N; n += kIiThreads) {
      float acc[kIiEnvs];
#pragma unroll
      for (int e = 0; e < kIiEnvs; ++e) acc[e] = 0.0f;
#pragma unroll 16
      for (int k = 0; k < K; ++k) {
        const float w = W[(size_t)k * N + n];
#pragma unroll
        for (int e = 0; e < kIiEnvs; ++e) acc[e] = __fmaf_rn(in[e * ldi + k], w, acc[e]);
      }
      const float b = bias[n];
#pragma unroll
      for (int e = 0; e < kIiEnvs; ++e) out[e * ldo + n] = ii_act(acc[e] + b, act);
    }
  } else {
    const int KS = kIiThreads / N;  // K slices
    const int Kc = (K + KS - 1) / KS;
    const int n = t % N, ks = t / N;
    if (ks < KS) {
      const int k0 = ks * Kc, k1 = min(K, k0 + Kc);
      float acc[kIiEnvs];
#pragma unroll
      for (int e = 0; e < kIiEnvs; ++e) acc[e] = 0.0f;
#pragma unroll 16
      for (int k = k0; k < k1; ++k) {
        const float w = W[(size_t)k * N + n];
#pragma unroll
        for (int e = 0; e < kIiEnvs; ++e) acc[e] = __fmaf_rn(in[e * ldi + k], w, acc[e]);
      }
#pragma unroll
      for (int e = 0; e < kIiEnvs; ++e) part[(ks * kIiEnvs + e) * N + n] = acc[e];
    }
    __syncthreads();
    for (int q = t; q < kIiEnvs * N; q += kIiThreads) {
      const int e = q / N, c = q - e * N;
      float s = 0.0f;
      for (int j = 0; j < KS; ++j) s += part[(j * kIiEnvs + e) * N + c];
      out[e * ldo + c] = ii_act(s + bias[c], act);
    }
  }
  __syncthreads();
}

// PREP: also CRoots::prepare for the workgroup's envs (prepare_root, lzm_tree.h) from the policy
// logits just written — the collect step's root preparation without a launch of its own.
template <bool PREP = false>
__global__ __launch_bounds__(kIiThreads) void initial_inference_kernel(IiArgs p, PrepareArgs q = PrepareArgs{}) {
  __shared__ float s_a[kIiEnvs * kIiMaxW], s_b[kIiEnvs * kIiMaxW], s_c[kIiEnvs * 256];
  __shared__ float s_part[kIiEnvs * kIiThreads];
  const int t = threadIdx.x;
  const int e0 = blockIdx.x * kIiEnvs;
  const int ne = min(kIiEnvs, p.B - e0);
  const int H = p.H;
  // PREP: the root's preparation inputs read at the start, into LDS / registers, so the tail below
  // is arithmetic and stores only (kIiEnvs == 1: the workgroup's root is e0)
  static_assert(!PREP || kIiEnvs == 1, "the fused preparation assumes one env per workgroup");
  __shared__ int s_leg[PREP ? kIiMaxW : 1];
  __shared__ float s_nz[PREP ? kIiMaxW : 1];
  int pr_n = 0, pr_tp = 0;
  float pr_rw = 0.0f;
  if (PREP) {
    const int A = q.A, cnt = q.count_in[e0];
    for (int j = t; j < A; j += kIiThreads) {
      s_leg[j] = cnt <= 0 ? j : (j < cnt ? q.legal_in[(size_t)e0 * A + j] : -1);
      s_nz[j] = q.noises ? q.noises[(size_t)e0 * A + j] : 0.0f;
    }
    pr_n = cnt <= 0 ? A : cnt;
    pr_tp = q.to_play[e0];
    pr_rw = q.rewards[e0];
  }
  for (int q = t; q < kIiEnvs * p.O; q += kIiThreads) {
    const int e = q / p.O, k = q - e * p.O;
    s_a[e * kIiMaxW + k] = e < ne ? p.obs[(size_t)(e0 + e) * p.O + k] : 0.0f;
  }
  __syncthreads();
  // representation: R1 (GELU) -> R2 -> SimNorm
  ii_dense(p.w[0], p.b[0], p.O, H, s_a, kIiMaxW, s_b, kIiMaxW, 2, s_part);
  ii_dense(p.w[1], p.b[1], H, H, s_b, kIiMaxW, s_a, kIiMaxW, 0, s_part);
  const int G = p.group;
  for (int q = t; q < kIiEnvs * (H / G); q += kIiThreads) {
    const int e = q / (H / G), g = q - e * (H / G);
    float *x = s_a + e * kIiMaxW + g * G;
    float m = x[0];
    for (int j = 1; j < G; ++j) m = fmaxf(m, x[j]);
    float s = 0.0f;
    for (int j = 0; j < G; ++j) s += expf(x[j] - m);
    for (int j = 0; j < G; ++j) x[j] = expf(x[j] - m) / s;
  }
  __syncthreads();
  for (int q = t; q < ne * H; q += kIiThreads) {
    const int e = q / H, k = q - e * H;
    p.latent[(size_t)(e0 + e) * H + k] = s_a[e * kIiMaxW + k];
  }
  // prediction: P1, P2 (ReLU) -> value head, policy head
  ii_dense(p.w[2], p.b[2], H, H, s_a, kIiMaxW, s_b, kIiMaxW, 1, s_part);
  ii_dense(p.w[3], p.b[3], H, H, s_b, kIiMaxW, s_a, kIiMaxW, 1, s_part);
  ii_dense(p.w[4], p.b[4], H, p.F, s_a, kIiMaxW, s_c, 256, 1, s_part);
  ii_dense(p.w[5], p.b[5], p.F, p.V, s_c, 256, s_b, kIiMaxW, 0, s_part);
  for (int q = t; q < ne * p.V; q += kIiThreads) {
    const int e = q / p.V, k = q - e * p.V;
    p.value[(size_t)(e0 + e) * p.V + k] = s_b[e * kIiMaxW + k];
  }
  ii_dense(p.w[6], p.b[6], H, p.F, s_a, kIiMaxW, s_c, 256, 1, s_part);
  ii_dense(p.w[7], p.b[7], p.F, p.A, s_c, 256, s_b, kIiMaxW, 0, s_part);
  for (int q = t; q < ne * p.A; q += kIiThreads) {
    const int e = q / p.A, k = q - e * p.A;
    p.policy[(size_t)(e0 + e) * p.A + k] = s_b[e * kIiMaxW + k];
  }
  if (PREP) {
    // CRoots::prepare for root i = e0, the same operations in the same order as prepare_root
    // (lzm_tree.h), with the legal list, noises and policy logits read from LDS
    const int i = e0, A = q.A, n = pr_n;
    for (int j = t; j < A; j += kIiThreads) q.legal[(size_t)i * A + j] = s_leg[j];
    if (t == 0) {
      q.nlegal[i] = n;
      const float *lg = s_b;  // this env's policy logits (e = 0)
      float pmax = kFloatMin;
      for (int j = 0; j < n; ++j) {
        const float l = lg[s_leg[j]];
        if (pmax < l) pmax = l;
      }
      float sum = 0.0f;
      for (int j = 0; j < n; ++j) sum += glibc_expf(lg[s_leg[j]] - pmax);
      const float f = q.noise_weight;
      for (int j = 0; j < n; ++j) {
        const int a = s_leg[j];
        float prior = glibc_expf(lg[a] - pmax) / sum;
        if (q.noises) prior = prior * (1 - f) + s_nz[j] * f;
        NodeStat c;
        c.visit = 0; c.value_sum = 0.0f; c.prior = prior; c.reward = 0.0f;
        q.stat[(size_t)(1 + a) * q.B + i] = c;
        NodeMeta cm;
        cm.latent = -1; cm.to_play = 0; cm.best = -1; cm.is_reset = 0;
        q.meta[(size_t)(1 + a) * q.B + i] = cm;
      }
      NodeStat r;
      r.visit = 1; r.value_sum = 0.0f; r.prior = 0.0f; r.reward = pr_rw;
      q.stat[i] = r;
      NodeMeta rm;
      rm.latent = 0; rm.to_play = pr_tp; rm.best = -1; rm.is_reset = 0;
      q.meta[i] = rm;
    }
  }
}

}  // namespace lzm
