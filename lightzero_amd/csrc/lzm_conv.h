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
#include <string.h>

#include "lzm_tree.h"

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
  int dyn, dres, rw, rb, pres, hw, hb, sc, bd, total;  // sc, bd: the split layout's scales and bounds (below)
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
  L.sc = L.bd = -1;
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
  float *out_r;          // [B][r_stride]: reward planes at [0, r_ch * 64)
  float *out_h;          // [B][h_ch * 64]
  int r_stride;          // floats per out_r row (r_ch * 64, or the EfficientZero LSTM input row)
  const float *hpool;    // nullable: EfficientZero LSTM hidden-state pool [.][B][H]; row x[b] of env b
  int H;                 // is copied to out_r[b][r_ch * 64 ..] (the [r | h] LSTM input row, no gather launch)
  int skip_dyn;          // 1: no dynamics conv — the input runs straight into the residual blocks, and no
                         // reward 1x1 (lzm_conv_resnet8_p: the representation network's 8 x 8 tail)
  int32_t *err;          // nullable: counts envs whose split activations left the fp16 range (split trunk)
  int32_t *xscale;       // with hpool: [B] the LSTM input row's scale exponent (lzm_lstm.h, ls_row_exp)
};

// [r | h] LSTM input row: the leaf's hidden state after the reward planes (every thread calls it)
__device__ __forceinline__ void trunk_copy_hidden(const ConvTrunkArgs &a, int b) {
  if (!a.hpool) return;
  const float4 *src = reinterpret_cast<const float4 *>(
      a.hpool + ((a.x ? (int64_t)max(a.x[b], 0) * a.B : 0) + b) * (int64_t)a.H);
  float4 *dst = reinterpret_cast<float4 *>(a.out_r + (int64_t)b * a.r_stride + a.r_ch * kCvPix);
  for (int k = threadIdx.x; k < (a.H >> 2); k += blockDim.x) dst[k] = src[k];
}

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
  trunk_copy_hidden(a, b);
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
  if (ch == 0) conv1_layer(buf(xi), a.w + L.rw, a.w + L.rb, a.r_ch, a.out_r + (int64_t)b * a.r_stride, lane, ph,
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

// ---------------------------------------------------------------------------------------------------
// Split trunk (precision 1, the default): the same network on v_mfma_f32_16x16x32_f16.
//
// Every f32 operand x is held as two fp16 terms x = h + l (h = fp16(x), l = fp16(x - h); the subtraction
// is exact). A product is summed from the three terms l_a h_b, h_a l_b, h_a h_b (the dropped l l term is
// <= 2^-22 relative). The fp16 matrix rate is 16x the f32 one (MI355X_MICROARCH.md constants: 16x16x32 16
// cycles vs 32x32x2 f32 64 cycles, 16x the K), so three products per K are 5.3x fewer matrix cycles than the
// exact-f32 kernel above.
//
// Range. fp16 holds |x| < 65504, and h + l keeps 22 significant bits only while l is a normal fp16 (|x| >=
// 2^-3); below that the split's error is an absolute 2^-25. So no operand is split as it is:
//   * weights: out channel c's row is packed as W_c 2^e_c, e_c = 14 - floor(log2 max_k |W_c,k|) (the row's
//     largest |w| in [2^14, 2^15)), clamped to +-kBxWExp; the epilogue multiplies by 2^-e_c, exactly;
//   * activations: each stored activation tensor (one env's 64 planes of one layer) as x 2^s, s = 14 -
//     floor(log2 bound), clamped to +-kBxAExp, with bound >= max |x| from what is known before the epilogue
//     stores it: the exact max of the layer's input M_in (each wave's max of its outputs meets the others'
//     in LDS at the barrier that follows every epilogue), the layer's packed bounds Wb = max_c sum_k |W_c,k|
//     and Bb = max_c |b_c| (the dynamics conv: max |actmap|), and the residual's exact max: bound = Wb M_in
//     + Bb (+ M_res). The input latent is scaled from its own exact max (one more barrier per step).
// A power of two commutes with fp16 and f32 rounding, so where the unscaled split was in range every term,
// product and sum is the same; elsewhere the split keeps its 22 bits down to 2^-17 below the tensor's
// bound. Every stored tensor's exact max is checked against its scale (max 2^s < 65504, and finite; only
// a non-finite value or one beyond ~2^114 can fail it) and a failure counts in the caller's error word
// (lzm_check_errors: LZM_ERR_RANGE). ReLUs propagate NaN (x < 0 ? 0 : x), as torch's do.
//
// Layout. Wave w owns out-channels 16w..16w+15 for all 64 pixels (four 16-pixel M tiles), so the four
// waves stream disjoint weights (221 KB per 3x3 layer per workgroup). K = tap-major (9 taps) x 64
// in-channels, in 18 chunks of 32. Activations live in LDS as the two fp16 planes of each buffer,
// [100 bordered positions][64 ch], 16-B chunk c of position ps stored at chunk c ^ ((ps % 10) & 7): the
// A-fragment reads (lane: pixel l&15 of the tile, channels 8(l>>4)..+7 of the chunk, one ds_read_b128)
// are then conflict-free for every tap (checked over the four lane groups of ds_read_b128).
// B fragments come from the host-packed [wave][chunk][term][lane][8 fp16] layout, one 1 KiB
// dwordx4 wave-load per term, a ring of AHEAD + 1 chunks issued AHEAD ahead.
constexpr int kBxTerms = 2;                        // fp16 terms per f32 operand (h, l)
constexpr int kBxComp = 100 * 64;                  // 16-bit elements per term plane
constexpr int kBxBuf = kBxTerms * kBxComp;         // per activation buffer (h, l planes); two buffers
constexpr int kBx3Frag = 4 * 18 * kBxTerms * 64 * 4;  // floats: [wave][chunk][term][lane][8 fp16]
constexpr int kBx1Frag = 2 * 2 * kBxTerms * 64 * 4;   // 1x1 64->32: [wave 0..1][chunk][term][lane][8 fp16]
constexpr int kBxBlock = 2 * kBx3Frag + 2 * kCvCh;
constexpr int kBxAhead = 3;  // default weight read-ahead (chunks)
// the EZ search's read-ahead: with fp16 terms (two uint4s per chunk) 5 chunks fit its registers and measured
// 2.49 -> 2.46 ms per Pong search; the Breakout search even at 2, 3, 4, 5 (profiles/r05/ab/ab_ahead.txt)
constexpr int kBxAheadEz = 5;
#ifndef LZM_RANGE_DIAG
#define LZM_RANGE_DIAG 0  // timing experiments only (results invalid): 1 = no max reduction, 2 = + no lane maxima,
                          // 3 = + max-form ReLU, 4 = + no scale multiplies
#endif
constexpr int kBxWExp = 24;   // weight-row scale exponents within +-24
constexpr int kBxAExp = 100;  // activation scale exponents within +-100: 2^-(e + s) stays a normal f32

typedef _Float16 bxh8 __attribute__((ext_vector_type(8)));
typedef float bxf4 __attribute__((ext_vector_type(4)));

// 2^n for |n| <= 126
__host__ __device__ inline float bx_pow2(int n) {
  const uint32_t u = (uint32_t)(127 + n) << 23;
  float x;
  memcpy(&x, &u, 4);
  return x;
}
// floor(log2 |x|) from the exponent field (0 and subnormals -> -127, inf / NaN -> 128)
__host__ __device__ inline int bx_ilog2(float x) {
  uint32_t u;
  memcpy(&u, &x, 4);
  return (int)((u >> 23) & 0xffu) - 127;
}
// the scale exponent that puts `bound` in [2^14, 2^15), clamped to +-lim
__host__ __device__ inline int bx_scale_exp(float bound, int lim) {
  const int s = 14 - bx_ilog2(bound);
  return s < -lim ? -lim : (s > lim ? lim : s);
}

// the scale exponent of an EfficientZero LSTM input row [reward planes | h] from the exact max of its reward
// planes (|h| < 1: the bound is max(M_r, 1); lzm_lstm.h)
__host__ __device__ inline int ls_row_exp(float reward_max) {
  return bx_scale_exp(reward_max > 1.f || reward_max != reward_max ? reward_max : 1.f, kBxAExp);
}

// the trunk's split: x = h + l, h = fp16(x), l = fp16(x - h) (x - h exact in f32), round to nearest even
__host__ __device__ inline void bx_split2(float x, uint16_t &h, uint16_t &l) {
  const _Float16 hh = (_Float16)x;
  const _Float16 ll = (_Float16)(x - (float)hh);
  h = __builtin_bit_cast(uint16_t, hh);
  l = __builtin_bit_cast(uint16_t, ll);
}

__host__ __device__ inline ConvTrunkLayout conv_trunk_layout_p(int n_dres, int n_pres, int precision) {
  if (precision == 0) return conv_trunk_layout(n_dres, n_pres);
  ConvTrunkLayout L;
  int o = 0;
  L.dyn = o; o += kBx3Frag;
  L.dres = o; o += n_dres * kBxBlock;
  L.rw = o; o += kBx1Frag;
  L.rb = o; o += 32;
  L.pres = o; o += n_pres * kBxBlock;
  L.hw = o; o += kBx1Frag;
  L.hb = o; o += 32;
  const int n3 = 1 + 2 * (n_dres + n_pres);
  L.sc = o; o += (n3 + 2) * 64;  // 2^-e_c per layer: the 3x3 layers in order, the reward 1x1, the head 1x1
  L.bd = o; o += (n3 + 2) * 4;   // {Wb, Bb, 0, 0} per layer, same order
  L.total = o;
  return L;
}

__device__ __forceinline__ bxh8 bx_ash(uint4 u) { return __builtin_bit_cast(bxh8, u); }

// Weight ring of one wave: RING chunks x the terms (one uint4 per lane each).
template <int AHEAD>
struct BxRing {
  uint4 w[AHEAD + 1][kBxTerms];
};

template <int AHEAD, int DIAG>
__device__ __forceinline__ void bx_load_w(BxRing<AHEAD> &r, const uint4 *__restrict__ wf, int s, int lane) {
#pragma unroll
  for (int q = 0; q < kBxTerms; ++q)
    r.w[s % (AHEAD + 1)][q] = DIAG == 1 ? uint4{(uint32_t)(lane + s), 1u, 2u, 3u} : wf[(s * kBxTerms + q) * 64 + lane];
}

// a conv's first chunks of weights; issued early (before the previous layer's epilogue and barrier)
template <int NCH, int AHEAD, int DIAG>
__device__ __forceinline__ void bx_prefetch(BxRing<AHEAD> &r, const uint4 *__restrict__ wf, int lane) {
#pragma unroll
  for (int s = 0; s < (NCH < AHEAD ? NCH : AHEAD); ++s) bx_load_w<AHEAD, DIAG>(r, wf, s, lane);
}

struct BxNoHook {
  __device__ void operator()(int) const {}
};

// one convolution for this wave's 16 out-channels x 64 pixels: NCH = 18 chunks (3x3) or 2 (1x1), its
// first AHEAD chunks already in the ring (bx_prefetch). DIAG = 1: no weight loads (timing
// experiments only, results invalid). Software pipeline, in issue order (the scheduling barriers keep
// the compiler from sinking loads next to their first use): weights of chunk s + AHEAD, activations
// of chunk s + 1, then chunk s's 12 MFMAs. hook(s): a little VALU work in chunk s's MFMA shadow (the range
// bookkeeping's wave reduction, one butterfly step per chunk).
template <int NCH, int AHEAD, int DIAG, class Hook = BxNoHook>
__device__ __forceinline__ void bx_conv(const uint16_t *in, const uint4 *__restrict__ wf, BxRing<AHEAD> &r, int lane,
                                        bxf4 (&acc)[4], const Hook &hook = Hook()) {
  uint4 a[2][4][kBxTerms];
  const int px = lane & 7, g = lane >> 4;
  // lane's pixel in tile t: p = 16t + (lane & 15), plane row py = 2t + ((lane >> 3) & 1), column px; tap
  // (dy, dx) reads bordered position (py + dy) * 10 + px + dx
  const int lbase = ((lane >> 3) & 1) * 10 + px;
  auto load_a = [&](int s) {
    const int tap = NCH == 2 ? 4 : s >> 1, j = NCH == 2 ? s : s & 1;
    const int dy = tap / 3, dx = tap % 3;
    const int chunk = ((4 * j + g) ^ (px + dx)) & 7;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int ps = lbase + (2 * t + dy) * 10 + dx;
#pragma unroll
      for (int q = 0; q < kBxTerms; ++q)
        a[s & 1][t][q] = *reinterpret_cast<const uint4 *>(in + q * kBxComp + ps * 64 + chunk * 8);
    }
  };
  load_a(0);
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = bxf4{0.f, 0.f, 0.f, 0.f};
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int s = 0; s < NCH; ++s) {
    if (s + AHEAD < NCH) bx_load_w<AHEAD, DIAG>(r, wf, s + AHEAD, lane);
    if (s + 1 < NCH) load_a(s + 1);
    const uint4 *w = r.w[s % (AHEAD + 1)];
    const uint4(&x)[4][kBxTerms] = a[s & 1];
    // small terms first: l_a h_b, h_a l_b, h_a h_b
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bx_ash(x[t][1]), bx_ash(w[0]), acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bx_ash(x[t][0]), bx_ash(w[1]), acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bx_ash(x[t][0]), bx_ash(w[0]), acc[t], 0, 0, 0);
    hook(s);
    // issue the next chunks' loads in the MFMA gaps (an MFMA holds the vector issue for half its
    // cycles): weights first (they have the longest way), then one activation read per MFMA
    const int nw = (s + AHEAD < NCH && DIAG != 1) ? kBxTerms : 0, na = s + 1 < NCH ? 4 * kBxTerms : 0;
#pragma unroll
    for (int k = 0; k < nw; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read
    }
#pragma unroll
    for (int k = 0; k < na; ++k) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
    }
#pragma unroll
    for (int k = 0; k < 12 - nw - na; ++k) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Accumulator (t, r) of a lane is out-channel c = 16 wave + (lane & 15) at pixel
// p = 16t + 4 (lane >> 4) + r: plane row 2t + (lane >> 5), column 4 ((lane >> 4) & 1) + r. The same lane
// owns the same (c, p) in every layer, so a residual block's input stays in that lane's registers
// (exact f32) and is added in the block's second epilogue without an LDS round trip.
__device__ __forceinline__ int bx_ep_pos(int lane, int t, int r) {
  return (2 * t + (lane >> 5) + 1) * 10 + 4 * ((lane >> 4) & 1) + r + 1;
}

// 3x3 epilogue: v = relu(acc f + bias [+ amap] [+ xres]) (f = 2^-(e_c + s_in): the weight row's and the input's
// scales undone) -> the split planes of `out` as v 2^s_out (so = 2^s_out); KEEP: xres = v. Returns the max of
// this lane's v as unsigned bits (v >= +0 or NaN: a NaN of either sign above every finite value) for the output's
// range bookkeeping (RELU only).
// RELU = false: store acc as is (the input latent's staging; f = 1, bias 0)
template <bool RELU = true>
__device__ __forceinline__ uint32_t bx_epilogue3(const bxf4 (&acc)[4], uint16_t *out, float f, float bc, bool use_am,
                                                 const float4 (&am)[4], float (&xres)[16], bool add_res, bool keep,
                                                 float so, int lane, int c) {
  typedef float bxf2 __attribute__((ext_vector_type(2)));
  typedef _Float16 bxb2 __attribute__((ext_vector_type(2)));
  const int cb = c >> 3, odd = lane & 1;
  uint32_t mx = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float x = RELU ? (LZM_RANGE_DIAG >= 4 ? acc[t][r] + bc : __fmaf_rn(acc[t][r], f, bc)) : acc[t][r];
      if (use_am) x += r == 0 ? am[t].x : r == 1 ? am[t].y : r == 2 ? am[t].z : am[t].w;
      if (add_res) x += xres[4 * t + r];
      // relu: NaN stays NaN, -0 becomes +0, so every output's bits order as unsigned integers with a NaN of either
      // sign above +inf (the range bookkeeping's max needs no masking)
      if (RELU) x = LZM_RANGE_DIAG >= 3 ? (x > 0.f ? x : 0.f) : (x <= 0.f ? 0.f : x);
      if (keep) xres[4 * t + r] = x;
      v[r] = x;
    }
    if (LZM_RANGE_DIAG < 2)
      mx = max(max(mx, __float_as_uint(v[0])), max(max(__float_as_uint(v[1]), __float_as_uint(v[2])),
                                                     __float_as_uint(v[3])));
    // lanes 2j, 2j + 1 hold channels c, c + 1 (one dword of a plane row): per pixel pair (2k, 2k + 1)
    // the even lane writes pixel 2k's dword and the odd lane pixel 2k + 1's, after one DPP swap
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const float send = odd ? v[2 * k] : v[2 * k + 1];
      const float recv = __builtin_bit_cast(
          float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, send), 0xB1, 0xF, 0xF, false));  // quad_perm 1,0,3,2
      const bxf2 pr = (odd ? bxf2{recv, v[2 * k + 1]} : bxf2{v[2 * k], recv}) * (LZM_RANGE_DIAG >= 4 ? 1.f : so);
      const bxb2 h = __builtin_convertvector(pr, bxb2);
      const bxb2 l = __builtin_convertvector(pr - __builtin_convertvector(h, bxf2), bxb2);
      const int r = 2 * k + odd;
      const int ps = bx_ep_pos(lane, t, r);
      // swizzle key (ps % 10) & 7 = column + 1; the pair's dword at channel c & ~1
      const int o = ps * 64 + (((cb ^ (4 * ((lane >> 4) & 1) + r + 1)) & 7) << 3) + (c & 6);
      *reinterpret_cast<bxb2 *>(out + o) = h;
      *reinterpret_cast<bxb2 *>(out + kBxComp + o) = l;
    }
  }
  return mx;
}

// the layers' bounds {Wb, Bb, 0, 0} into LDS once per launch (read per layer without a scalar load in the way of
// the LDS counter); nl = n3 + 2 <= kBxMaxLayers
constexpr int kBxMaxLayers = 1 + 2 * 16 + 2;
__device__ __forceinline__ void bx_stage_bounds(float4 *s_bd, const float *w, const ConvTrunkLayout &L, int nl, int tid,
                                                int nthreads) {
  for (int i = tid; i < nl; i += nthreads) s_bd[i] = reinterpret_cast<const float4 *>(w + L.bd)[i];
}

// Range bookkeeping of one workgroup's trunk (every wave holds the same copy): the exact max |x| of the
// current layer input and of the current block input, the input buffer's scale exponent, a sticky failure.
// Per layer: the epilogue writes each lane's max of its outputs (bits) to LDS, unreduced; after the barrier
// every lane reads four of the 256 and the wave reduces them inside the next convolution, one butterfly step per
// weight chunk (bx_range_step as bx_conv's hook), where each step's operand is a chunk old: the max of a layer's
// output is first needed for the NEXT layer's output scale.
struct BxRange {
  float m_in, m_blk;
  int s_in, bad;
  uint32_t m;  // the reduction in flight
  uint4 lm;    // this lane's four of the previous epilogue's 256 lane maxima (read after the barrier)
};

// this wave's max (lane maxima as bits) into its LDS slot; read back after the next barrier (bx_read_max)
__device__ __forceinline__ void bx_post_max(uint32_t *slot, uint32_t mx, int wv, int lane) {
  mx = (uint32_t)xor_max((int)mx);  // (bits of |x| <= 0x7fffffff: the signed max is the unsigned one)
  if (lane == 0) slot[wv] = mx;
}
__device__ __forceinline__ float bx_read_max(const uint32_t *slot) {
  const uint4 v = *reinterpret_cast<const uint4 *>(slot);
  return __uint_as_float(max(max(v.x, v.y), max(v.z, v.w)));
}
// the max |x| of a latent of this lane's 16 values; one barrier (every thread)
__device__ __forceinline__ float bx_latent_max(const float (&xres)[16], uint32_t *slot, int wv, int lane) {
  uint32_t mx = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) mx = max(mx, __float_as_uint(xres[j]) & 0x7fffffffu);
  bx_post_max(slot, mx, wv, lane);
  __syncthreads();
  return bx_read_max(slot);
}
// the input latent of exact max m: its scale
__device__ __forceinline__ BxRange bx_range_input(float m) {
  BxRange rg;
  rg.m_in = rg.m_blk = m;
  rg.s_in = bx_scale_exp(m, kBxAExp);
  rg.bad = !(m * bx_pow2(rg.s_in) < 65504.f);
  rg.m = 0u;
  rg.lm = uint4{0u, 0u, 0u, 0u};
  return rg;
}
// the output scale of a 3x3 layer from its packed bounds bd = {Wb, Bb}; res: + the block input (the dynamics
// conv: + the latent). A block's first conv makes its input the block input.
__device__ __forceinline__ int bx_layer_scale(const float4 bd, bool res, BxRange &rg) {
  if (!res) rg.m_blk = rg.m_in;
  float bound = bd.x * rg.m_in + bd.y;
  if (res) bound += rg.m_blk;
  return bx_scale_exp(bound, kBxAExp);
}
// after the barrier that follows an epilogue storing at scale s_out: this lane's four lane maxima (slots[256])
__device__ __forceinline__ void bx_range_fetch(BxRange &rg, const uint32_t *slots, int s_out, int lane) {
  rg.lm = reinterpret_cast<const uint4 *>(slots)[lane];
  rg.s_in = s_out;
}
// step s of the reduction (s = 0 .. 7; bx_conv's hook calls it per chunk): then the layer input's exact max,
// checked against its scale (lane maxima are unsigned bits of outputs >= +0 or NaN: bx_epilogue3)
__device__ __forceinline__ void bx_range_step(BxRange &rg, int s) {
  if (LZM_RANGE_DIAG >= 1) return;
  if (s == 0) rg.m = max(max(rg.lm.x, rg.lm.y), max(rg.lm.z, rg.lm.w));
  if (s == 1) rg.m = max(rg.m, (uint32_t)xor_partner<32>((int)rg.m));
  if (s == 2) rg.m = max(rg.m, (uint32_t)xor_partner<16>((int)rg.m));
  if (s == 3) rg.m = max(rg.m, (uint32_t)xor_partner<8>((int)rg.m));
  if (s == 4) rg.m = max(rg.m, (uint32_t)xor_partner<4>((int)rg.m));
  if (s == 5) rg.m = max(rg.m, (uint32_t)xor_partner<2>((int)rg.m));
  if (s == 6) rg.m = max(rg.m, (uint32_t)xor_partner<1>((int)rg.m));
  if (s == 7) {
    const float M = __uint_as_float(rg.m);
    rg.bad |= !(M * bx_pow2(rg.s_in) < 65504.f);
    rg.m_in = M;
  }
}
__device__ __forceinline__ void bx_range_reduce(BxRange &rg) {
#pragma unroll
  for (int s = 0; s < 8; ++s) bx_range_step(rg, s);
}
// The form the kernels use: each wave reduces its epilogue's lane maxima (unsigned bits of outputs >= +0 or NaN:
// a NaN of either sign above +inf) to one word in its LDS slot before the barrier that follows every epilogue,
// and after it every lane takes the layer output's exact max from the four slots (bx_range_take). (Measured
// against the staged reduction above — one butterfly step per weight chunk inside the next convolution —
// Breakout search 1.665 vs 1.687 ms, Pong even; profiles/r06/range/.)
__device__ __forceinline__ void bx_post_umax(uint32_t *slot, uint32_t mx, int wv, int lane) {
  mx = max(mx, (uint32_t)xor_partner<32>((int)mx));
  mx = max(mx, (uint32_t)xor_partner<16>((int)mx));
  mx = max(mx, (uint32_t)xor_partner<8>((int)mx));
  mx = max(mx, (uint32_t)xor_partner<4>((int)mx));
  mx = max(mx, (uint32_t)xor_partner<2>((int)mx));
  mx = max(mx, (uint32_t)xor_partner<1>((int)mx));
  if (lane == 0) slot[wv] = mx;
}
// after the barrier that follows an epilogue storing at scale s_out (slot: its four wave maxima): the layer
// output's exact max, checked against its scale; it is the next layer's input
__device__ __forceinline__ void bx_range_take(BxRange &rg, const uint32_t *slot, int s_out) {
  rg.s_in = s_out;
  if (LZM_RANGE_DIAG >= 1) return;
  const float M = bx_read_max(slot);
  rg.bad |= !(M * bx_pow2(s_out) < 65504.f);
  rg.m_in = M;
}

// 1x1 layer (<= 32 out channels, waves 0 and 1): relu(conv x inv[c] 2^-s_in + b) -> global [c][p]
// (SC1: 16-B sc1 buffer stores, for planes another CU reads in the same launch); returns the lane's max |v| (bits)
template <int DIAG, bool SC1 = false>
__device__ __forceinline__ uint32_t bx_conv1_layer(const uint16_t *in, const float *__restrict__ wl,
                                               const float *__restrict__ bias, const float *__restrict__ inv,
                                               float sinv, int nch, float *dst, int lane, int wv) {
  BxRing<2> r1;
  const uint4 *wf = reinterpret_cast<const uint4 *>(wl) + wv * 2 * kBxTerms * 64;
  bx_prefetch<2, 2, DIAG>(r1, wf, lane);
  const int c = 16 * wv + (lane & 15);
  const float bc = c < nch ? bias[c] : 0.f, f = c < nch ? inv[c] * sinv : 0.f;
  bxf4 acc[4];
  bx_conv<2, 2, DIAG>(in, wf, r1, lane, acc);
  if (c >= nch) return 0u;
  auto relu = [&](float x) { x = __fmaf_rn(x, f, bc); return x < 0.f ? 0.f : x; };
  uint32_t mx = 0;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const float4 v = float4{relu(acc[t][0]), relu(acc[t][1]), relu(acc[t][2]), relu(acc[t][3])};
    mx = max(max(mx, __float_as_uint(v.x) & 0x7fffffffu),
             max(__float_as_uint(v.y) & 0x7fffffffu, max(__float_as_uint(v.z) & 0x7fffffffu,
                                                         __float_as_uint(v.w) & 0x7fffffffu)));
    if constexpr (SC1) {
      typedef unsigned u4v __attribute__((ext_vector_type(4)));
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, nch * kCvPix * 4, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), rs, (c * kCvPix + 16 * t + 4 * (lane >> 4)) * 4,
                                             0, 16);
    } else {
      *reinterpret_cast<float4 *>(dst + c * kCvPix + 16 * t + 4 * (lane >> 4)) = v;
    }
  }
  return mx;
}

// The 3x3 layers in order: 0 = dynamics conv, then two per residual block (dynamics blocks, then
// prediction blocks); the reward 1x1 follows layer 2 n_dres, the head 1x1 the last one. Activations
// ping-pong between two LDS buffers (layer i reads buffer i & 1): residuals travel in registers.
__device__ __forceinline__ int bx_layer_off(const ConvTrunkLayout &L, int n_dres, int i) {
  if (i == 0) return L.dyn;
  const int j = i - 1, base = j < 2 * n_dres ? L.dres : L.pres, k = j < 2 * n_dres ? j : j - 2 * n_dres;
  return base + (k >> 1) * kBxBlock + (k & 1) * (kBx3Frag + kCvCh);
}

// zero the 36 border positions of both buffers' term planes ([buffer][term][border position][16-B chunk])
__device__ __forceinline__ void bx_zero_borders(uint4 *lds4, int tid, int nthreads) {
  for (int k = tid; k < 2 * kBxTerms * 36 * 8; k += nthreads) {
    const int ch = k & 7, bp = (k >> 3) % 36, plane = k / (36 * 8);
    const int ps = bp < 10 ? bp : bp < 20 ? 80 + bp : (1 + ((bp - 20) >> 1)) * 10 + ((bp - 20) & 1) * 9;
    lds4[(plane * kBxComp + ps * 64) / 8 + ch] = uint4{0u, 0u, 0u, 0u};
  }
}

template <int AHEAD>
__global__ __launch_bounds__(kCvThreads) __attribute__((amdgpu_waves_per_eu(1, 1))) void conv_trunk_bx_kernel(
    ConvTrunkArgs a) {
  extern __shared__ uint4 bx_lds4[];
  __shared__ uint32_t s_mx[4], s_rmx[2], s_wm[2][4];
  __shared__ float4 s_bd[kBxMaxLayers];
  uint16_t *lds = reinterpret_cast<uint16_t *>(bx_lds4);
  auto buf = [&](int i) { return lds + i * kBxBuf; };
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int c = 16 * wv + (lane & 15);
  const ConvTrunkLayout L = conv_trunk_layout_p(a.n_dres, a.n_pres, 1);
  const int n3 = 1 + 2 * a.n_dres + 2 * a.n_pres;
  const float *inv = a.w + L.sc;
  const float4 *bd = s_bd;
  bx_stage_bounds(s_bd, a.w, L, n3 + 2, tid, kCvThreads);  // (ordered by the first barrier)
  auto layer_w = [&](int i) { return a.w + bx_layer_off(L, a.n_dres, i); };
  auto wave_stream = [&](const float *w) { return reinterpret_cast<const uint4 *>(w) + wv * 18 * kBxTerms * 64; };
  const int i0 = a.skip_dyn ? 1 : 0;  // the first layer run (skip_dyn: the first residual block's)
  BxRing<AHEAD> ring;
  bx_prefetch<18, AHEAD, 0>(ring, wave_stream(layer_w(i0)), lane);
  // the input latent: this lane's 16 values in registers (the dynamics residual, exact f32) ...
  const float *src = a.pool + ((a.x ? (int64_t)max(a.x[b], 0) * a.B : 0) + b) * (int64_t)(kCvCh * kCvPix);
  float xres[16];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const float4 v = *reinterpret_cast<const float4 *>(src + c * kCvPix + 16 * t + 4 * (lane >> 4));
    xres[4 * t] = v.x; xres[4 * t + 1] = v.y; xres[4 * t + 2] = v.z; xres[4 * t + 3] = v.w;
  }
  trunk_copy_hidden(a, b);
  BxRange rg = bx_range_input(bx_latent_max(xres, s_mx, wv, lane));
  // ... split into buffer 0 from those registers by the epilogue's store path (interior), while the
  // 36 border positions of both buffers are zeroed (disjoint addresses: one barrier)
  {
    bxf4 in4[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) in4[t] = bxf4{xres[4 * t], xres[4 * t + 1], xres[4 * t + 2], xres[4 * t + 3]};
    const float4 no_am[4] = {};
    bx_epilogue3<false>(in4, buf(i0 & 1), 1.f, 0.f, false, no_am, xres, false, false, bx_pow2(rg.s_in), lane, c);
  }
  bx_zero_borders(bx_lds4, tid, kCvThreads);
  __syncthreads();
  for (int i = i0; i < n3; ++i) {
    const float *w = layer_w(i);
    const bool second = i > 0 && ((i - 1) & 1);  // a block's second conv: + residual, new block input
    // epilogue operands first (vmcnt counts in order: they must not queue behind the next prefetch)
    const float bc = i ? w[kBx3Frag + c] : 0.f;
    const float4 bdi = bd[i];
    const float wsc = inv[i * 64 + c];
    float4 am[4] = {};
    if (i == 0) {
      const float4 *amap = reinterpret_cast<const float4 *>(a.actmap + ((int64_t)a.action[b] * kCvCh + c) * kCvPix);
#pragma unroll
      for (int t = 0; t < 4; ++t) am[t] = amap[4 * t + (lane >> 4)];
    }
    bxf4 acc[4];
    bx_conv<18, AHEAD, 0>(buf(i & 1), wave_stream(w), ring, lane, acc);
    if (i + 1 < n3) bx_prefetch<18, AHEAD, 0>(ring, wave_stream(layer_w(i + 1)), lane);
    const int s_out = bx_layer_scale(bdi, i == 0 || second, rg);
    bx_post_umax(s_wm[i & 1],
                 bx_epilogue3(acc, buf((i + 1) & 1), wsc * bx_pow2(-rg.s_in), bc, i == 0, am, xres, i == 0 || second,
                              i == 0 || second, bx_pow2(s_out), lane, c),
                 wv, lane);
    __syncthreads();
    bx_range_take(rg, s_wm[i & 1], s_out);
    if (i == 2 * a.n_dres) {  // the next latent (registers, exact) and the reward planes
      float *dst = a.out_latent + (int64_t)b * kCvCh * kCvPix + c * kCvPix + 4 * (lane >> 4);
#pragma unroll
      for (int t = 0; t < 4; ++t)
        *reinterpret_cast<float4 *>(dst + 16 * t) = float4{xres[4 * t], xres[4 * t + 1], xres[4 * t + 2], xres[4 * t + 3]};
      if (!a.skip_dyn && wv < 2) {
        const uint32_t rm = bx_conv1_layer<0>(buf((i + 1) & 1), a.w + L.rw, a.w + L.rb, inv + n3 * 64,
                                              bx_pow2(-rg.s_in), a.r_ch, a.out_r + (int64_t)b * a.r_stride, lane, wv);
        bx_post_max(s_rmx, rm, wv, lane);
      }
    }
  }
  if (wv < 2)
    bx_conv1_layer<0>(buf(n3 & 1), a.w + L.hw, a.w + L.hb, inv + (n3 + 1) * 64, bx_pow2(-rg.s_in), a.h_ch,
                      a.out_h + (int64_t)b * a.h_ch * kCvPix, lane, wv);
  if (a.xscale) {  // the LSTM input row's scale (every wave reaches this barrier)
    __syncthreads();
    if (tid == 0) a.xscale[b] = ls_row_exp(__uint_as_float(max(s_rmx[0], s_rmx[1])));
  }
  if (rg.bad && tid == 0 && a.err) atomicAdd(a.err, 1);
}

// host packing for the split trunk (every weight row scaled, the layer's bounds). 3x3: W[64 out][64 in][9] ->
// [wave][chunk s][term][lane][8]: chunk s = 2 * tap + j, lane -> (out 16 * wave + (lane & 15), in 32 j + 8 (lane >>
// 4) + e); inv[64] = 2^-e_c; bd[0] = Wb
inline int bx_row_exp(const float *row, int n, double *l1) {
  float m = 0.f;
  double s = 0.0;
  for (int k = 0; k < n; ++k) {
    const float v = fabsf(row[k]);
    m = v > m ? v : m;
    s += v;
  }
  *l1 = s;
  return m > 0.f ? bx_scale_exp(m, kBxWExp) : 0;
}
// a float >= the double x (the bounds are upper bounds)
inline float bx_round_up(double x) { return (float)(x * (1.0 + 1e-6)); }

inline void bx_pack3(const float *W, float *outf, float *inv, float *bd) {
  uint16_t *out = reinterpret_cast<uint16_t *>(outf);
  int e[64];
  double wb = 0.0;
  for (int co = 0; co < 64; ++co) {
    double l1;
    e[co] = bx_row_exp(W + co * 64 * 9, 64 * 9, &l1);
    inv[co] = bx_pow2(-e[co]);
    wb = l1 > wb ? l1 : wb;
  }
  bd[0] = bx_round_up(wb);
  for (int w = 0; w < 4; ++w)
    for (int s = 0; s < 18; ++s)
      for (int lane = 0; lane < 64; ++lane)
        for (int el = 0; el < 8; ++el) {
          const int tap = s >> 1, j = s & 1, cin = 32 * j + 8 * (lane >> 4) + el, cout = 16 * w + (lane & 15);
          uint16_t t[kBxTerms];
          bx_split2(ldexpf(W[(cout * 64 + cin) * 9 + tap], e[cout]), t[0], t[1]);
          for (int q = 0; q < kBxTerms; ++q) out[(((w * 18 + s) * kBxTerms + q) * 64 + lane) * 8 + el] = t[q];
        }
}

// 1x1: W[n <= 32 out][64 in] -> [wave 0..1][chunk j][term][lane][8], zero columns past n
inline void bx_pack1(const float *W, int n, float *outf, float *inv, float *bd) {
  uint16_t *out = reinterpret_cast<uint16_t *>(outf);
  int e[32];
  double wb = 0.0;
  for (int co = 0; co < 32; ++co) {
    double l1 = 0.0;
    e[co] = co < n ? bx_row_exp(W + co * 64, 64, &l1) : 0;
    inv[co] = bx_pow2(-e[co]);
    wb = l1 > wb ? l1 : wb;
  }
  bd[0] = bx_round_up(wb);
  for (int w = 0; w < 2; ++w)
    for (int j = 0; j < 2; ++j)
      for (int lane = 0; lane < 64; ++lane)
        for (int el = 0; el < 8; ++el) {
          const int cin = 32 * j + 8 * (lane >> 4) + el, cout = 16 * w + (lane & 15);
          uint16_t t[kBxTerms] = {0, 0};
          if (cout < n) bx_split2(ldexpf(W[cout * 64 + cin], e[cout]), t[0], t[1]);
          for (int q = 0; q < kBxTerms; ++q) out[(((w * 2 + j) * kBxTerms + q) * 64 + lane) * 8 + el] = t[q];
        }
}

// max |b| over n biases (rounded up)
inline float bx_bias_bound(const float *b, int n) {
  double m = 0.0;
  for (int k = 0; k < n; ++k) m = fabs((double)b[k]) > m ? fabs((double)b[k]) : m;
  return bx_round_up(m);
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
