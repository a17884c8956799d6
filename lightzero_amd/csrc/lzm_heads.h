// lzm_heads.h — the MLP heads of the conv recurrent step in one launch (configs 3 and 5).
//
// After the convolutional trunk (lzm_conv.h) the reference evaluates, per env
// (muzero_model.py:505-530 reward head, common.py:854-881 prediction heads; EfficientZero adds
// the LSTM and its value-prefix BatchNorm, efficientzero_model.py:526-574):
//   reward hidden   rh = relu(W_rh1 r + b)            r: reward planes (MZ) or relu(BN(h_lstm)) (EZ)
//   reward logits   W_rh2 rh + b                      (support Vr)
//   value hidden    vh = relu(W_v1 hd[value planes] + b),  policy hidden ph = relu(W_p1 hd[policy planes] + b)
//   value logits    W_v2 vh + b (support Vv),  policy logits W_p2 ph + b (A)
// with every BatchNorm folded on the host (conv_infer.py). As separate GEMMs these are six tiny
// launches plus two ReLU passes per simulation. Here the grid is (env blocks of 2) x (3 heads):
// 384 workgroups at B = 256 (8.7 us; blocks of 4: 13 us), instead of one workgroup per 8 envs
// (32 workgroups measured 38.6 us, L2-latency bound on the serial weight stream). Every thread
// issues all of its weight loads (128 + 96 registers) before the first wait, so the weights cost one
// L2 round trip, not one per loop batch (13.0 -> see DESIGN.md 6.3). A workgroup stages its head's
// input rows in LDS and runs both layers with fp32 FMAs (f32 MFMA has the same
// rate on gfx950, and 4 rows would fill a 16-row tile a quarter). Weights come from L2 in layouts
// built at fold time so every wave-instruction reads contiguous bytes:
//   w1t  [3 heads][8 parts][32 k4][32 cols][4]: hidden column c of a head over its K range
//        part * 128 + 4 k4 .. +3 (zero past the head's K)
//   w2t  [32 k][N2 cols]: output column j (reward Vr | value Vv | policy A) over its head's hidden
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lzm_tree.h"

namespace lzm {

constexpr int kHdEnvs = 2;     // envs per workgroup
constexpr int kHdThreads = 256;
constexpr int kHdParts = 8;    // K split of the first layer, one per 32-lane half wave
constexpr int kHdKMax = 1024;  // K per head (8 parts of 128)
constexpr int kHdRMax = 1024;  // reward input width
constexpr int kHdHMax = 2048;  // head planes width
constexpr int kHdCols = 3;     // output columns per thread: supports up to 768

struct HeadsArgs {
  int B, Kr, Khd;
  const float *r, *r_scale, *r_shift;  // r [B][Kr]; optional relu(r * scale + shift) (EZ)
  const float *hd;                     // [B][Khd]
  int src[3], off[3], K[3];            // per head: input (0: r, 1: hd), its offset and width
  const float *w1t, *b1;               // see above; b1 [96]
  const float *w2t, *b2;               // [32][N2], [N2]
  int Vr, Vv, A;
  float *reward, *value, *policy;      // [B][Vr], [B][Vv], [B][A]
  int32_t *norm_words;                 // optional: ensure_softmax verdict words (see below)
  int norm_nparts;                     // norm_parts(B) word pairs the consumer ANDs
  int head0;                           // first head of the grid's y range (1: prediction heads only)
  // lzm_conv_heads_prepare: the policy-head workgroups also prepare their envs' roots from the logits they
  // computed (CRoots::prepare, prepare_root: the root preparation launch folded in); A <= kHdThreads
  PrepareArgs prep;
  int prep_on;
};

__global__ __launch_bounds__(kHdThreads) void conv_heads_kernel(HeadsArgs p) {
  __shared__ float4 s_in4[kHdEnvs * kHdKMax / 4];
  __shared__ float s_part[kHdParts][kHdEnvs][32];
  __shared__ float s_hid[kHdEnvs][32];
  float *s_in = reinterpret_cast<float *>(s_in4);
  const int tid = threadIdx.x;
  const int head = blockIdx.y + p.head0;
  const int e0 = blockIdx.x * kHdEnvs;
  const int ne = min(kHdEnvs, p.B - e0);
  const int K = p.K[head];
  const bool from_r = p.src[head] == 0;
  const float *src = from_r ? p.r : p.hd;
  const int row = from_r ? p.Kr : p.Khd;
  const int part = tid >> 5, c = tid & 31;
  const bool part_live = part * 128 < K;
  // ---- every weight this thread needs, issued before anything waits (one L2 round trip instead of
  // one per unrolled batch): its 32 first-layer float4s and its output columns' 32-deep slices
  float4 w1[32];
  {
    const float4 *w = reinterpret_cast<const float4 *>(p.w1t) + ((size_t)(head * kHdParts + part) * 32) * 32 + c;
#pragma unroll
    for (int k4 = 0; k4 < 32; ++k4) w1[k4] = part_live ? w[(size_t)k4 * 32] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  }
  const int N2 = p.Vr + p.Vv + p.A;
  const int j0 = head == 0 ? 0 : (head == 1 ? p.Vr : p.Vr + p.Vv);
  const int wd = head == 0 ? p.Vr : (head == 1 ? p.Vv : p.A);
  float w2[kHdCols][32], b2[kHdCols];
#pragma unroll
  for (int cc = 0; cc < kHdCols; ++cc) {
    const int jj = tid + cc * kHdThreads;
    const bool live = jj < wd;
#pragma unroll
    for (int k = 0; k < 32; ++k) w2[cc][k] = live ? p.w2t[(size_t)k * N2 + j0 + jj] : 0.0f;
    b2[cc] = live ? p.b2[j0 + jj] : 0.0f;
  }
  // ---- stage this head's input rows (zero past K and past the batch): all four float4 loads of a
  // thread in flight together (a load-wait-store loop costs one memory latency per element)
  {
    constexpr int kQ = kHdEnvs * kHdKMax / 4 / kHdThreads;
    float4 v[kQ];
#pragma unroll
    for (int u = 0; u < kQ; ++u) {
      const int q = tid + u * kHdThreads, e = q / (kHdKMax / 4), k = 4 * (q - e * (kHdKMax / 4));
      v[u] = (e < ne && k < K) ? *reinterpret_cast<const float4 *>(src + (size_t)(e0 + e) * row + p.off[head] + k)
                               : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
#pragma unroll
    for (int u = 0; u < kQ; ++u) {
      const int q = tid + u * kHdThreads, e = q / (kHdKMax / 4), k = 4 * (q - e * (kHdKMax / 4));
      float4 x = v[u];
      if (from_r && p.r_scale && e < ne && k < K) {
        x.x = fmaxf(__fmaf_rn(x.x, p.r_scale[k], p.r_shift[k]), 0.0f);
        x.y = fmaxf(__fmaf_rn(x.y, p.r_scale[k + 1], p.r_shift[k + 1]), 0.0f);
        x.z = fmaxf(__fmaf_rn(x.z, p.r_scale[k + 2], p.r_shift[k + 2]), 0.0f);
        x.w = fmaxf(__fmaf_rn(x.w, p.r_scale[k + 3], p.r_shift[k + 3]), 0.0f);
      }
      s_in4[q] = x;
    }
  }
  __syncthreads();
  // ---- hidden layer: lane (part, c) sums its 128-wide K range for the workgroup's envs
  {
    const float *in = s_in + part * 128;
    float acc[kHdEnvs];
#pragma unroll
    for (int e = 0; e < kHdEnvs; ++e) acc[e] = 0.0f;
    if (part_live) {
#pragma unroll
      for (int k4 = 0; k4 < 32; ++k4) {
        const float4 q = w1[k4];
#pragma unroll
        for (int e = 0; e < kHdEnvs; ++e) {
          const float4 x = *reinterpret_cast<const float4 *>(in + e * kHdKMax + 4 * k4);
          acc[e] = __fmaf_rn(x.x, q.x, acc[e]);
          acc[e] = __fmaf_rn(x.y, q.y, acc[e]);
          acc[e] = __fmaf_rn(x.z, q.z, acc[e]);
          acc[e] = __fmaf_rn(x.w, q.w, acc[e]);
        }
      }
    }
#pragma unroll
    for (int e = 0; e < kHdEnvs; ++e) s_part[part][e][c] = acc[e];
  }
  __syncthreads();
  if (tid < kHdEnvs * 32) {
    const int e = tid >> 5, cc = tid & 31;
    float s = 0.0f;
#pragma unroll
    for (int q = 0; q < kHdParts; ++q) s += s_part[q][e][cc];
    s_hid[e][cc] = fmaxf(s + p.b1[head * 32 + cc], 0.0f);
  }
  __syncthreads();
  // ---- output layer: kHdCols columns of this head per thread, 32-deep dot per env
  float *out = head == 0 ? p.reward : (head == 1 ? p.value : p.policy);
  const bool prep = p.prep_on && head == 2;  // (block-uniform)
  __shared__ float s_lg[kHdEnvs][kHdThreads];
  float rsum[kHdEnvs];  // this thread's share of each row's sum (verdict words below)
#pragma unroll
  for (int e = 0; e < kHdEnvs; ++e) rsum[e] = 0.0f;
#pragma unroll
  for (int cc = 0; cc < kHdCols; ++cc) {
    const int jj = tid + cc * kHdThreads;
    if (jj >= wd) break;
    float acc[kHdEnvs];
#pragma unroll
    for (int e = 0; e < kHdEnvs; ++e) acc[e] = 0.0f;
#pragma unroll
    for (int k = 0; k < 32; ++k) {
#pragma unroll
      for (int e = 0; e < kHdEnvs; ++e) acc[e] = __fmaf_rn(s_hid[e][k], w2[cc][k], acc[e]);
    }
    for (int e = 0; e < ne; ++e) out[(size_t)(e0 + e) * wd + jj] = acc[e] + b2[cc];
#pragma unroll
    for (int e = 0; e < kHdEnvs; ++e) rsum[e] += acc[e] + b2[cc];
    if (prep && cc == 0) {
#pragma unroll
      for (int e = 0; e < kHdEnvs; ++e) s_lg[e][jj] = acc[e] + b2[cc];
    }
  }
  if (prep) {
    __syncthreads();
    if (tid < ne) prepare_root(p.prep, e0 + tid, s_lg[tid]);
  }
  // ensure_softmax's verdict (scaling_transform.py:36-62) for the reward and value rows this
  // workgroup wrote, in the word layout normalized_check_kernel uses (lzm_kernels.hip): word pair q,
  // head h is 0 iff a row of that head fails allclose(sum, 1); pairs nb.. are set to 1 here so the
  // consumer's AND over norm_parts(B) pairs sees exactly these verdicts. Saves one launch per step.
  if (p.norm_words && head < 2) {
    __shared__ float s_sum[kHdEnvs][kHdThreads / 64];
#pragma unroll
    for (int e = 0; e < kHdEnvs; ++e) {
      const float v = xor_sum(rsum[e]);
      if ((tid & 63) == 0) s_sum[e][tid >> 6] = v;
    }
    __syncthreads();
    if (tid == 0) {
      int ok = 1;
      for (int e = 0; e < ne; ++e) {
        const float sm = (s_sum[e][0] + s_sum[e][1]) + (s_sum[e][2] + s_sum[e][3]);
        if (!(fabsf(sm - 1.0f) <= 1e-5f + 1e-5f)) ok = 0;
      }
      const int nb = gridDim.x;
      p.norm_words[2 * blockIdx.x + head] = ok;
      if (nb + (int)blockIdx.x < p.norm_nparts) p.norm_words[2 * (nb + blockIdx.x) + head] = 1;
    }
  }
}

}  // namespace lzm
