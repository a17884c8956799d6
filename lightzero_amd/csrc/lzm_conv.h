// lzm_conv.h — the convolutional trunk of the recurrent step for the Atari configs (BASELINE.json
// configs 3 and 5: MuZeroModel / EfficientZeroModel with a 64 x 8 x 8 latent), one workgroup per env.
//
// Per simulation the search calls recurrent_inference (mcts_ctree.py:291-298 / :776-790); its
// convolutional part, with every eval-mode BatchNorm folded (lightzero_amd/conv_infer.py), is
//   dynamics  (muzero_model.py:505-530, efficientzero_model.py:526-574):
//     X1 = relu(conv3x3(latent, Wd) + actmap[action] + latent)        actmap holds the action
//          planes' contribution and the folded bias (constant planes -> a per-action [64][8][8] map)
//     n_dres x basic block: Y = relu(conv3x3(X) + b1); X = relu(conv3x3(Y) + b2 + X)   -> next latent
//     reward planes R = relu(conv1x1(next latent) + br)                [r_ch <= 32][8][8]
//   prediction (common.py:854-881):
//     n_pres x basic block on the next latent;  head planes H = relu(conv1x1(.) + bh)
//     (the value and policy 1x1 convolutions stacked: [h_ch <= 32][8][8])
// This kernel runs all of it for one env in one workgroup, with the activations in LDS, and writes
// the next latent (straight into the search's latent pool slot), R and H; the head MLPs / LSTM stay
// batched GEMMs over the envs.
//
// Each 3x3 convolution is a GEMM  [64 pixels] x [576 = 9 taps x 64 in-channels] -> [64 out-channels]
// on v_mfma_f32_32x32x2_f32 (f32 in, f32 accumulate — the exact-f32 matrix path of gfx950, at the
// f32 peak rate): 4 waves, wave w owns pixels 32*(w&1).. and out-channels 32*(w>>1)..; A (pixels x
// k) is read straight from the zero-bordered 10 x 10 planes in LDS (no im2col), B (k x out) comes
// from the host-packed fragment layout, one 1 KiB dwordx4 wave-load per 4 MFMAs, all 72 of a layer
// issued up front. Epilogue (bias, residual from LDS, action map, ReLU) on the accumulators.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lzm {

constexpr int kCvThreads = 256;
constexpr int kCvCh = 64;               // latent channels
constexpr int kCvPix = 64;              // 8 x 8 plane
constexpr int kCvCS = 101;              // LDS floats per channel: 10 x 10 zero-bordered plane + 1 (bank spread)
constexpr int kCvBuf = kCvCh * kCvCS;   // one activation buffer
constexpr int kCv3Frag = 2 * 72 * 64 * 4;  // 3x3 64->64: [out half][step/4][lane][4]
constexpr int kCv1Frag = 8 * 64 * 4;       // 1x1 64->32: [step/4][lane][4]
constexpr int kCvBlock = 2 * kCv3Frag + 2 * kCvCh;  // basic block: W1 frag, b1, W2 frag, b2

typedef float cvf16 __attribute__((ext_vector_type(16)));

struct ConvTrunkLayout {
  int dyn, dres, rw, rb, pres, hw, hb, total;
};

__host__ __device__ inline ConvTrunkLayout conv_trunk_layout(int n_dres, int n_pres) {
  ConvTrunkLayout L;
  int o = 0;
  L.dyn = o; o += kCv3Frag;
  L.dres = o; o += n_dres * kCvBlock;
  L.rw = o; o += kCv1Frag;
  L.rb = o; o += 32;
  L.pres = o; o += n_pres * kCvBlock;
  L.hw = o; o += kCv1Frag;
  L.hb = o; o += 32;
  L.total = o;
  return L;
}

struct ConvTrunkArgs {
  int B, n_dres, n_pres, r_ch, h_ch;
  const float *w;        // conv_trunk_layout floats (lzm_conv_trunk_prepare)
  const float *actmap;   // [A][64][64]: action planes' conv + folded bias of the dynamics conv
  const float *pool;     // input latents: pool[x[b]][b] if x, else pool[b]   ([.][B][4096])
  const int32_t *x;      // nullable
  const int32_t *action; // [B]
  float *out_latent;     // [B][4096]
  float *out_r;          // [B][r_ch * 64]
  float *out_h;          // [B][h_ch * 64]
};

// one 3x3 (TAPS = 9) or 1x1 (TAPS = 1) convolution of the LDS planes `in` for this wave's tile
template <int TAPS>
__device__ __forceinline__ cvf16 conv_tile(const float *in, const float4 *__restrict__ wf, int lane, int abase) {
  // weights: a ring of three taps (8 dwordx4 = 32 MFMA steps each), loads issued two taps ahead;
  // the scheduling barriers keep the compiler from sinking them next to their first use
  float4 wr[3][8];
#pragma unroll
  for (int t = 0; t < (TAPS < 2 ? TAPS : 2); ++t) {
#pragma unroll
    for (int q = 0; q < 8; ++q) wr[t][q] = wf[(t * 8 + q) * 64 + lane];
    __builtin_amdgcn_sched_barrier(0);  // issue order = consumption order (vmcnt counts in order)
  }
  cvf16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int tap = 0; tap < TAPS; ++tap) {
    if (tap + 2 < TAPS) {
#pragma unroll
      for (int q = 0; q < 8; ++q) wr[(tap + 2) % 3][q] = wf[((tap + 2) * 8 + q) * 64 + lane];
      __builtin_amdgcn_sched_barrier(0);
    }
    const int toff = TAPS == 9 ? (tap / 3) * 10 + (tap % 3) : 11;
    float a[32];
#pragma unroll
    for (int c2 = 0; c2 < 32; ++c2) a[c2] = in[abase + 2 * c2 * kCvCS + toff];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c2 = 0; c2 < 32; ++c2) {
      const float4 wq = wr[tap % 3][c2 >> 2];
      const float b = (c2 & 3) == 0 ? wq.x : (c2 & 3) == 1 ? wq.y : (c2 & 3) == 2 ? wq.z : wq.w;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[c2], b, acc, 0, 0, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  return acc;
}

// accumulator element r of lane -> (out channel within the 32-wide half, pixel within the 32-pixel half)
__device__ __forceinline__ int cv_row(int lane, int r) { return 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3); }

__device__ __forceinline__ int cv_plane(int p) { return ((p >> 3) + 1) * 10 + (p & 7) + 1; }

// 3x3 layer: out = relu(conv(in) + bias [+ res] [+ amap]) into LDS
__device__ __forceinline__ void conv3_layer(const float *in, float *out, const float *res, const float *__restrict__ wl,
                                            const float *__restrict__ bias, const float *__restrict__ amap, int lane,
                                            int ph, int ch, int abase) {
  cvf16 acc = conv_tile<9>(in, reinterpret_cast<const float4 *>(wl) + ch * 72 * 64, lane, abase);
  const int c = ch * 32 + (lane & 31);
  const float bc = bias ? bias[c] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int p = ph * 32 + cv_row(lane, r);
    const int o = c * kCvCS + cv_plane(p);
    float v = acc[r] + bc;
    if (amap) v += amap[c * kCvPix + p];
    if (res) v += res[o];
    out[o] = v > 0.f ? v : 0.f;
  }
}

// 1x1 layer (<= 32 out channels, waves of the first out-channel half): relu(conv + b) -> global [c][p]
__device__ __forceinline__ void conv1_layer(const float *in, const float *__restrict__ wl, const float *__restrict__ bias,
                                            int nch, float *dst, int lane, int ph, int abase) {
  cvf16 acc = conv_tile<1>(in, reinterpret_cast<const float4 *>(wl), lane, abase);
  const int c = lane & 31;
  if (c >= nch) return;
  const float bc = bias[c];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int p = ph * 32 + cv_row(lane, r);
    const float v = acc[r] + bc;
    dst[c * kCvPix + p] = v > 0.f ? v : 0.f;
  }
}

__global__ __launch_bounds__(kCvThreads) __attribute__((amdgpu_waves_per_eu(1, 1))) void conv_trunk_kernel(
    ConvTrunkArgs a) {
  extern __shared__ float cv_lds[];
  auto buf = [&](int i) { return cv_lds + i * kCvBuf; };
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int ph = wv & 1, ch = wv >> 1;
  // A-operand base: lane supplies row (pixel) ph*32 + lane%32 and k-parity lane/32 (in-channel 2*c2 + hi)
  const int pA = ph * 32 + (lane & 31);
  const int abase = (lane >> 5) * kCvCS + (pA >> 3) * 10 + (pA & 7);
  const ConvTrunkLayout L = conv_trunk_layout(a.n_dres, a.n_pres);
  for (int i = tid; i < 3 * kCvBuf; i += kCvThreads) cv_lds[i] = 0.f;  // zero borders
  __syncthreads();
  // x = -1 (a search-with-reuse root that needs no inference): any row will do, its output is unused
  const float *src = a.pool + ((a.x ? (int64_t)max(a.x[b], 0) * a.B : 0) + b) * (int64_t)(kCvCh * kCvPix);
  for (int i = tid; i < kCvCh * kCvPix / 4; i += kCvThreads) {
    const float4 v = reinterpret_cast<const float4 *>(src)[i];
    const int c = (4 * i) >> 6, p = (4 * i) & 63;
    float *d = buf(0) + c * kCvCS + cv_plane(p);
    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;  // p..p+3 share a plane row
  }
  __syncthreads();
  // dynamics conv: X1 = relu(conv(X0) + actmap[a] + X0)
  const float *amap = a.actmap + (int64_t)a.action[b] * kCvCh * kCvPix;
  conv3_layer(buf(0), buf(1), buf(0), a.w + L.dyn, nullptr, amap, lane, ph, ch, abase);
  __syncthreads();
  int xi = 1, yi = 2, zi = 0;  // block input, temp, output
  for (int k = 0; k < a.n_dres; ++k) {
    const float *wb = a.w + L.dres + k * kCvBlock;
    conv3_layer(buf(xi), buf(yi), nullptr, wb, wb + kCv3Frag, nullptr, lane, ph, ch, abase);
    __syncthreads();
    conv3_layer(buf(yi), buf(zi), buf(xi), wb + kCv3Frag + kCvCh, wb + 2 * kCv3Frag + kCvCh, nullptr, lane, ph, ch,
                abase);
    __syncthreads();
    const int t = xi; xi = zi; zi = yi; yi = t;
  }
  // next latent: to the pool slot, and reward planes
  {
    float *dst = a.out_latent + (int64_t)b * kCvCh * kCvPix;
    const float *s = buf(xi);
    for (int i = tid; i < kCvCh * kCvPix; i += kCvThreads) dst[i] = s[(i >> 6) * kCvCS + cv_plane(i & 63)];
  }
  if (ch == 0) conv1_layer(buf(xi), a.w + L.rw, a.w + L.rb, a.r_ch, a.out_r + (int64_t)b * a.r_ch * kCvPix, lane, ph,
                           abase);
  for (int k = 0; k < a.n_pres; ++k) {
    const float *wb = a.w + L.pres + k * kCvBlock;
    conv3_layer(buf(xi), buf(yi), nullptr, wb, wb + kCv3Frag, nullptr, lane, ph, ch, abase);
    __syncthreads();
    conv3_layer(buf(yi), buf(zi), buf(xi), wb + kCv3Frag + kCvCh, wb + 2 * kCv3Frag + kCvCh, nullptr, lane, ph, ch,
                abase);
    __syncthreads();
    const int t = xi; xi = zi; zi = yi; yi = t;
  }
  if (ch == 0) conv1_layer(buf(xi), a.w + L.hw, a.w + L.hb, a.h_ch, a.out_h + (int64_t)b * a.h_ch * kCvPix, lane, ph,
                           abase);
}

// host packing: natural layouts -> fragment layouts
// 3x3: W[64 out][64 in][9]  ->  [half][s4][lane][q], step s = 4*s4 + q = tap*32 + c2,
//      lane -> (in = 2*c2 + lane/32, out = 32*half + lane%32)
inline void conv_pack3(const float *W, float *out) {
  for (int half = 0; half < 2; ++half)
    for (int s = 0; s < 288; ++s)
      for (int lane = 0; lane < 64; ++lane) {
        const int tap = s / 32, c2 = s % 32, cin = 2 * c2 + (lane >> 5), cout = 32 * half + (lane & 31);
        out[((half * 72 + s / 4) * 64 + lane) * 4 + (s & 3)] = W[(cout * 64 + cin) * 9 + tap];
      }
}

// 1x1: W[n <= 32 out][64 in] -> [s4][lane][q], step s = c2, zero columns past n
inline void conv_pack1(const float *W, int n, float *out) {
  for (int s = 0; s < 32; ++s)
    for (int lane = 0; lane < 64; ++lane) {
      const int cin = 2 * s + (lane >> 5), cout = lane & 31;
      out[((s / 4) * 64 + lane) * 4 + (s & 3)] = cout < n ? W[cout * 64 + cin] : 0.f;
    }
}

}  // namespace lzm
