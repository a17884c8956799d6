// lzm_repr.h — the representation network's downsampling stages of the Atari configs (BASELINE.json configs 3
// and 5) on the split-bf16 matrix path: initial_inference's DownSample (lzero/model/common.py:164-265), with
// every eval-mode BatchNorm folded into the convolution in front of it (lightzero_amd/conv_infer.py):
//
//   L1  y = relu(conv3x3_s2(obs, W1) + b1)                         obs [C <= 7][64][64] -> [32][32][32]
//   L2  t = relu(conv3x3(y) + b)          L3  y = relu(conv3x3(t) + b + y)           (resblocks1)
//   L4  d = relu(conv3x3_s2(y, W1) + b1), s = conv3x3_s2(y, W3)    [32][32][32] -> 2 x [64][16][16]
//   L5  x = relu(conv3x3(d, W2) + b2 + s)                          (the downsample block)
//   L6  t = relu(conv3x3(x) + b)          L7  x = relu(conv3x3(t) + b + x)           (resblocks2)
//   avg_pool 3x3 / 2 (pad 1, count_include_pad) -> [64][8][8] NCHW, the 8 x 8 tail's input (lzm_conv_resnet8_p)
//
// One launch per convolution, activations NHWC f32 in HBM (the whole [B][32][32][32] stage is 33 MB at B = 256:
// it stays in the Infinity Cache between layers). Each convolution is an implicit GEMM: rows = out channels
// (the MFMA A operand: the folded weights, held in REGISTERS for the whole launch), columns = output pixels
// (the B operand: read from an LDS image of the input halo), K = 9 taps x in-channels in chunks of 32, on
// v_mfma_f32_16x16x32_bf16 with every f32 operand split into three bf16 terms (six products per K: f32-level
// error, the trunk's scheme, lzm_conv.h). A persistent grid (one 4-wave workgroup per CU) walks 64-pixel
// output tiles; the next tile's halo is loaded into registers before the current tile's MFMAs and written to
// the other LDS buffer after them.
//
// LDS image of a halo, per bf16 term: [channel group g = 8 channels][position][8 bf16], a group's plane padded
// to a multiple of 16 positions. A B-fragment read (lane: pixel l & 15 of a 16-pixel tile, channel group
// g0 + (l >> 4)) touches 16 consecutive positions per group, so every ds_read_b128 lane group hits 16
// distinct 16-B bank slots. Stride-2 convolutions store the halo's even and odd columns apart, which makes
// their reads consecutive too. The first layer (C <= 7 input channels, NCHW) stages an im2col tile instead:
// K = tap * C + channel, zero-padded to 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lzm_conv.h"

namespace lzm {

constexpr int kRpThreads = 512;  // 8 waves: two per SIMD

struct ReprConvArgs {
  int B, ntiles, cin_obs;  // cin_obs: first layer's input channels (MODE 2)
  const float *in;         // NHWC [B][HIN][HIN][CIN] (MODE 2: NCHW obs [B][cin_obs][64][64])
  const float *w;          // fragments [out tile][chunk][term][lane][8 bf16] (repr_pack)
  const float *bias;       // [COUT] (MODE 1: [64], the first half's)
  const float *res;        // nullable: NHWC residual of the output's shape
  float *out;              // NHWC [B][HOUT][HOUT][COUT] (MODE 1: the first 64 channels)
  float *out2;             // MODE 1: the shortcut's 64 channels, NHWC
};

// Geometry of one layer: WOUT-wide output rows, 64-pixel tiles of TR rows; halo HR x HC (bordered), LDS row
// pitch ROWP (stride 2: even columns, then odd ones), group plane NPP positions (a multiple of 16).
template <int CIN, int COUT, int STRIDE, int WOUT, int MODE>
struct ReprGeom {
  // output pixels per tile: 128 for the 32-channel layers (two pixel tiles per wave), 64 otherwise
  static constexpr int PX = COUT == 32 ? 128 : 64;
  static constexpr int TR = PX / WOUT;
  static constexpr int HR = MODE == 2 ? 1 : (TR - 1) * STRIDE + 3;
  static constexpr int HC = MODE == 2 ? PX : (WOUT - 1) * STRIDE + 3;
  static constexpr int HC2 = (HC + 1) / 2;
  static constexpr int ROWP = STRIDE == 2 && MODE != 2 ? 2 * HC2 : HC;
  static constexpr int NP = HR * ROWP;
  static constexpr int NPP = (NP + 15) / 16 * 16;
  static constexpr int CG = MODE == 2 ? 8 : CIN / 8;                  // channel groups (MODE 2: 64 K / 8)
  static constexpr int NCH = MODE == 2 ? 2 : 9 * (CIN / 32);          // K chunks of 32
  static constexpr int OT = COUT / 16;                                // out-channel tiles
  // 8 waves, one out tile each: 2 out tiles -> a pixel tile per wave; 4 -> all 4 pixel tiles over half of K
  // (KS = 2: K split, partial sums exchanged through LDS); 8 -> all 4 pixel tiles, all of K
  static constexpr int KS = OT == 4 ? 2 : 1;
  static constexpr int PTW = OT == 2 ? PX / 64 : PX / 16;             // pixel tiles per wave
  static constexpr int NCW = NCH / KS;                                // K chunks per wave
  static_assert(OT == 2 || OT == 4 || OT == 8, "out tiles");
  static_assert(NCH % KS == 0, "K split");
  static constexpr int TERM = CG * NPP * 8;                           // bf16 per term image
  static constexpr int BUF = 3 * TERM;                                // bf16 per halo buffer
  static constexpr int PPW = MODE == 2 ? 64 : 64 / CG;                // positions per wave-instruction
  // staging items (position, group): 64 per wave-instruction, PPW consecutive positions x CG groups
  static constexpr int ITEMS = MODE == 2 ? PX * 8 : (HR * HC + PPW - 1) / PPW * 64;
  static constexpr int IPT = (ITEMS + kRpThreads - 1) / kRpThreads;  // per thread
};

// the LDS position of halo (row hr, bordered column hc)
template <class G, int STRIDE>
__device__ __forceinline__ int rp_pos(int hr, int hc) {
  if constexpr (STRIDE == 2) return hr * G::ROWP + (hc & 1) * G::HC2 + (hc >> 1);
  else return hr * G::ROWP + hc;
}

// staging item q of a tile -> (LDS position, channel group); false past the last item
template <class G, int STRIDE, int MODE>
__device__ __forceinline__ bool rp_item(int q, int &hr, int &hc, int &g) {
  if (q >= G::ITEMS) return false;
  if constexpr (MODE == 2) {
    hr = 0;
    hc = q % G::PX;  // pixel of the tile
    g = q / G::PX;
    return true;
  }
  // lanes: PPW consecutive halo positions (global: whole NHWC rows, coalesced; LDS: distinct bank slots per
  // 8-lane write group) x the CG channel groups
  const int lin = (q >> 6) * G::PPW + (q & 63) % G::PPW;
  if (lin >= G::HR * G::HC) return false;
  g = (q & 63) / G::PPW;
  hr = lin / G::HC;
  hc = lin % G::HC;
  return true;
}

// x where ok, else +0 (a bit mask: no select of addresses for the compiler to turn into a scratch array)
__device__ __forceinline__ float4 rp_keep(bool ok, float4 x) {
  const uint32_t m = ok ? 0xffffffffu : 0u;
  return float4{__uint_as_float(__float_as_uint(x.x) & m), __uint_as_float(__float_as_uint(x.y) & m),
                __uint_as_float(__float_as_uint(x.z) & m), __uint_as_float(__float_as_uint(x.w) & m)};
}

// load this thread's staging items of tile `tile` into registers (8 f32 per item). Branch-free: every item
// loads from a clamped in-bounds address and selects zero where it lies outside the image (the halo border),
// so the registers stay registers (no private-array stores under divergent control flow) and the loads stay
// in flight until rp_store
template <int CIN, int COUT, int STRIDE, int WOUT, int MODE>
__device__ __forceinline__ void rp_load(const ReprConvArgs &a, int tile, float4 (&v)[ReprGeom<CIN, COUT, STRIDE, WOUT, MODE>::IPT][2]) {
  typedef ReprGeom<CIN, COUT, STRIDE, WOUT, MODE> G;
  constexpr int HIN = WOUT * STRIDE;
  constexpr int TPI = (WOUT / G::TR);  // tiles per image (square output: WOUT rows)
  const int b = tile / TPI, r0 = (tile % TPI) * G::TR;
#pragma unroll
  for (int i = 0; i < G::IPT; ++i) {
    int hr = 0, hc = 0, g = 0;
    const bool item = rp_item<G, STRIDE, MODE>(threadIdx.x + i * kRpThreads, hr, hc, g);
    if constexpr (MODE == 2) {
      // im2col: pixel hc of the tile (row r0 + hc / WOUT, column hc % WOUT), K = 8 g .. 8 g + 7 = tap * C + c
      const int oy = r0 + hc / WOUT, ox = hc % WOUT;
      float e[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 8 * g + j, tap = k / a.cin_obs, c = k % a.cin_obs;
        const int iy = 2 * oy + tap / 3 - 1, ix = 2 * ox + tap % 3 - 1;
        const bool ok = item && tap < 9 && iy >= 0 && iy < 64 && ix >= 0 && ix < 64;
        const float x = a.in[ok ? (((int64_t)b * a.cin_obs + c) * 64 + iy) * 64 + ix : 0];
        e[j] = __uint_as_float(__float_as_uint(x) & (ok ? 0xffffffffu : 0u));
      }
      v[i][0] = float4{e[0], e[1], e[2], e[3]};
      v[i][1] = float4{e[4], e[5], e[6], e[7]};
    } else {
      const int iy = r0 * STRIDE - 1 + hr, ix = hc - 1;
      const bool ok = item && iy >= 0 && iy < HIN && ix >= 0 && ix < HIN;
      const float4 *src = reinterpret_cast<const float4 *>(
          a.in + (ok ? (((int64_t)b * HIN + iy) * HIN + ix) * CIN + 8 * g : 0));
      v[i][0] = rp_keep(ok, src[0]);
      v[i][1] = rp_keep(ok, src[1]);
    }
  }
}

// split the loaded items into the three bf16 term images of an LDS halo buffer
template <int CIN, int COUT, int STRIDE, int WOUT, int MODE>
__device__ __forceinline__ void rp_store(uint16_t *buf, const float4 (&v)[ReprGeom<CIN, COUT, STRIDE, WOUT, MODE>::IPT][2]) {
  typedef ReprGeom<CIN, COUT, STRIDE, WOUT, MODE> G;
  typedef __bf16 b8 __attribute__((ext_vector_type(8)));
  typedef float f8 __attribute__((ext_vector_type(8)));
#pragma unroll
  for (int i = 0; i < G::IPT; ++i) {
    int hr, hc, g;
    if (!rp_item<G, STRIDE, MODE>(threadIdx.x + i * kRpThreads, hr, hc, g)) continue;
    const int pos = MODE == 2 ? hc : rp_pos<G, STRIDE>(hr, hc);
    const f8 x = f8{v[i][0].x, v[i][0].y, v[i][0].z, v[i][0].w, v[i][1].x, v[i][1].y, v[i][1].z, v[i][1].w};
    const b8 h = __builtin_convertvector(x, b8);
    const f8 r1 = x - __builtin_convertvector(h, f8);
    const b8 m = __builtin_convertvector(r1, b8);
    const b8 l = __builtin_convertvector(r1 - __builtin_convertvector(m, f8), b8);
    const int o = (g * G::NPP + pos) * 8;
    *reinterpret_cast<b8 *>(buf + o) = h;
    *reinterpret_cast<b8 *>(buf + G::TERM + o) = m;
    *reinterpret_cast<b8 *>(buf + 2 * G::TERM + o) = l;
  }
}

template <int CIN, int COUT, int STRIDE, int WOUT, int MODE>
__global__ __launch_bounds__(kRpThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void repr_conv_kernel(
    ReprConvArgs a) {
  typedef ReprGeom<CIN, COUT, STRIDE, WOUT, MODE> G;
  extern __shared__ uint4 rp_lds4[];
  uint16_t *lds = reinterpret_cast<uint16_t *>(rp_lds4);
  float *xscr = reinterpret_cast<float *>(lds + 2 * G::BUF);  // K-split partial sums
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // this wave's out tile, first pixel tile and K half
  const int ot = G::OT == 2 ? (wv & 1) : (G::OT == 4 ? (wv & 3) : wv);
  const int pt0 = G::OT == 2 ? (wv >> 1) * G::PTW : 0;
  const int kh = G::KS == 2 ? (wv >> 2) : 0;
  // the weights of that out tile over its K chunks, three terms: registers for the whole launch
  uint4 wr[G::NCW][3];
#pragma unroll
  for (int s = 0; s < G::NCW; ++s)
#pragma unroll
    for (int q = 0; q < 3; ++q)
      wr[s][q] = reinterpret_cast<const uint4 *>(a.w)[((ot * G::NCH + kh * G::NCW + s) * 3 + q) * 64 + lane];
  // out channels 4 (lane >> 4) .. + 3 of the tile; the dual layer's upper half is the shortcut (no bias)
  constexpr int COUT_T = MODE == 1 ? COUT / 2 : COUT;  // channels of one output tensor
  constexpr int HOUT = WOUT, TPI = HOUT / G::TR;
  int ch = 16 * ot + 4 * (lane >> 4);
  const bool sc = MODE == 1 && ch >= COUT_T;
  float *dst = sc ? a.out2 : a.out;
  if (sc) ch -= COUT_T;
  const float4 bias = sc ? float4{0.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const float4 *>(a.bias + ch);
  float4 v[G::IPT][2];
  int tile = blockIdx.x;
  if (tile < a.ntiles) {
    rp_load<CIN, COUT, STRIDE, WOUT, MODE>(a, tile, v);
    rp_store<CIN, COUT, STRIDE, WOUT, MODE>(lds, v);
  }
  __syncthreads();
  for (int it = 0; tile < a.ntiles; ++it, tile += gridDim.x) {
    const uint16_t *cur = lds + (it & 1) * G::BUF;
    const int nxt = tile + gridDim.x;
    if (nxt < a.ntiles) rp_load<CIN, COUT, STRIDE, WOUT, MODE>(a, nxt, v);  // in flight during the MFMAs
    const int b = tile / TPI, r0 = (tile % TPI) * G::TR;
    // the epilogue's residual, issued now (its latency hides behind the MFMAs): one float4 per pixel tile this
    // wave finishes (K split: 2, the tiles 2 kh + j), none for the dual layer
    constexpr int NRES = MODE == 1 ? 1 : (G::KS == 2 ? 2 : G::PTW);
    float4 rres[NRES];
#pragma unroll
    for (int j = 0; j < NRES; ++j) {
      const int p = G::KS == 2 ? 2 * kh + j : j;
      const int px = 16 * (pt0 + p) + (lane & 15);
      const int64_t e = (((int64_t)b * HOUT + r0 + px / WOUT) * WOUT + px % WOUT) * COUT_T + ch;
      rres[j] = (MODE != 1 && a.res) ? *reinterpret_cast<const float4 *>(a.res + e) : float4{0.f, 0.f, 0.f, 0.f};
    }
    bxf4 acc[G::PTW];
#pragma unroll
    for (int p = 0; p < G::PTW; ++p) acc[p] = bxf4{0.f, 0.f, 0.f, 0.f};
    // B fragments of chunk s for the wave's pixel tiles (lane: pixel 16 (pt0 + p) + (lane & 15) of the tile,
    // output row px / WOUT, column px % WOUT; channel group 4 j + (lane >> 4))
    auto load_x = [&](int s, uint4 (&x)[G::PTW][3]) {
      const int sg = kh * G::NCW + s;  // chunk within the layer's K
      const int tap = MODE == 2 ? 0 : sg / (CIN / 32), j = MODE == 2 ? sg : sg % (CIN / 32);
      const int dy = tap / 3, dx = tap % 3, g = 4 * j + (lane >> 4);
#pragma unroll
      for (int p = 0; p < G::PTW; ++p) {
        const int px = 16 * (pt0 + p) + (lane & 15);
        int pos;
        if constexpr (MODE == 2) pos = px;
        else pos = rp_pos<G, STRIDE>((px / WOUT) * STRIDE + dy, (px % WOUT) * STRIDE + dx);
#pragma unroll
        for (int q = 0; q < 3; ++q)
          x[p][q] = *reinterpret_cast<const uint4 *>(cur + q * G::TERM + (g * G::NPP + pos) * 8);
      }
    };
    // software pipeline: chunk s + 1's LDS reads issued before chunk s's MFMAs (the scheduling barrier keeps
    // the compiler from hoisting every chunk's reads to the top, which would need 9 x the fragment registers)
    uint4 xa[G::PTW][3], xb[G::PTW][3];
    load_x(0, xa);
#pragma unroll
    for (int s = 0; s < G::NCW; ++s) {
      uint4(&xc)[G::PTW][3] = (s & 1) ? xb : xa;
      uint4(&xn)[G::PTW][3] = (s & 1) ? xa : xb;
      if (s + 1 < G::NCW) load_x(s + 1, xn);
      const uint4(&w)[3] = wr[s];
#pragma unroll
      for (int p = 0; p < G::PTW; ++p) {
        // small terms first: w_l x_h, w_h x_l, w_m x_m, w_m x_h, w_h x_m, w_h x_h
        bxf4 c = acc[p];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx_as(w[2]), bx_as(xc[p][0]), c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx_as(w[0]), bx_as(xc[p][2]), c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx_as(w[1]), bx_as(xc[p][1]), c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx_as(w[1]), bx_as(xc[p][0]), c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx_as(w[0]), bx_as(xc[p][1]), c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bx_as(w[0]), bx_as(xc[p][0]), c, 0, 0, 0);
        acc[p] = c;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // K split: the K-half-0 wave finishes pixel tiles 0-1, the K-half-1 wave tiles 2-3; each hands the other
    // its partial sums of the other two through LDS
    if constexpr (G::KS == 2) {
      float4 *mine = reinterpret_cast<float4 *>(xscr + ((ot * 2 + (1 - kh)) * 64 + lane) * 8);
      const bxf4 g0 = kh ? acc[0] : acc[2], g1 = kh ? acc[1] : acc[3];
      mine[0] = float4{g0[0], g0[1], g0[2], g0[3]};
      mine[1] = float4{g1[0], g1[1], g1[2], g1[3]};
      __syncthreads();
      const float4 *theirs = reinterpret_cast<const float4 *>(xscr + ((ot * 2 + kh) * 64 + lane) * 8);
      const float4 q0 = theirs[0], q1 = theirs[1];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const float4 q = (p & 1) ? q1 : q0;
        if ((p >> 1) == kh) {
          acc[p][0] += q.x; acc[p][1] += q.y; acc[p][2] += q.z; acc[p][3] += q.w;
        }
      }
    }
    // epilogue: acc[p][r] = out channel ch + r at pixel 16 (pt0 + p) + (lane & 15)
#pragma unroll
    for (int p = 0; p < G::PTW; ++p) {
      if (G::KS == 2 && (p >> 1) != kh) continue;  // (the K-split partner's tiles)
      const int px = 16 * (pt0 + p) + (lane & 15);
      const int64_t e = (((int64_t)b * HOUT + r0 + px / WOUT) * WOUT + px % WOUT) * COUT_T + ch;
      float4 y = float4{acc[p][0] + bias.x, acc[p][1] + bias.y, acc[p][2] + bias.z, acc[p][3] + bias.w};
      if (!sc) {
        if (a.res) {
          const float4 rr = rres[MODE == 1 ? 0 : (G::KS == 2 ? (p & 1) : p)];
          y.x += rr.x; y.y += rr.y; y.z += rr.z; y.w += rr.w;
        }
        y.x = fmaxf(y.x, 0.f); y.y = fmaxf(y.y, 0.f); y.z = fmaxf(y.z, 0.f); y.w = fmaxf(y.w, 0.f);
      }
      *reinterpret_cast<float4 *>(dst + e) = y;
    }
    if (nxt < a.ntiles) rp_store<CIN, COUT, STRIDE, WOUT, MODE>(lds + ((it + 1) & 1) * G::BUF, v);
    __syncthreads();
  }
}

// avg_pool2d(3, 2, padding 1, count_include_pad) of NHWC [B][16][16][64] -> NCHW [B][64][8][8]: one workgroup per
// image, the 64 KiB image staged through LDS (coalesced float4 reads; positions padded to 65 floats so the
// pooling reads of consecutive output columns fall in different banks), NCHW written coalesced
__global__ __launch_bounds__(256) void repr_avgpool_kernel(const float *__restrict__ in, float *__restrict__ out, int B) {
  __shared__ float img[256 * 65];
  const int b = blockIdx.x, tid = threadIdx.x;
  const float4 *src = reinterpret_cast<const float4 *>(in + (size_t)b * 16384);
#pragma unroll 4
  for (int q = tid; q < 4096; q += 256) {
    const float4 v = src[q];
    float *d = img + (q >> 4) * 65 + (q & 15) * 4;
    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
  }
  __syncthreads();
  float *dst = out + (size_t)b * 4096;
#pragma unroll 4
  for (int o = tid; o < 4096; o += 256) {
    const int c = o >> 6, y = (o >> 3) & 7, x = o & 7;
    float s = 0.f;
    for (int dy = -1; dy <= 1; ++dy) {
      const int iy = 2 * y + dy;
      if (iy < 0 || iy >= 16) continue;
      for (int dx = -1; dx <= 1; ++dx) {
        const int ix = 2 * x + dx;
        if (ix < 0 || ix >= 16) continue;
        s += img[(iy * 16 + ix) * 65 + c];
      }
    }
    dst[o] = s / 9.0f;
  }
}

// ---- host side: packing
// A-operand fragments of one convolution: W [cout][cin][3][3] (folded) -> [out tile][chunk][term][lane][8 bf16],
// lane -> out channel 16 tile + (lane & 15), K = 8 (lane >> 4) + e within the chunk; chunk s = tap * (cin / 32)
// + j with K -> in channel 32 j + ..., or (first layer, cin <= 7) chunk s with K = 32 s + ... = tap * cin + c.
// Two weights stacked (the dual layer: W [64] then W3 [64]) give cout = 128.
inline void repr_pack(const float *W, int cout, int cin, bool im2col, float *outf) {
  uint16_t *out = reinterpret_cast<uint16_t *>(outf);
  const int nch = im2col ? 2 : 9 * (cin / 32);
  for (int ot = 0; ot < cout / 16; ++ot)
    for (int s = 0; s < nch; ++s)
      for (int lane = 0; lane < 64; ++lane)
        for (int e = 0; e < 8; ++e) {
          const int co = 16 * ot + (lane & 15), k = 8 * (lane >> 4) + e;
          float wv = 0.f;
          if (im2col) {
            const int kk = 32 * s + k, tap = kk / cin, c = kk % cin;
            if (tap < 9) wv = W[(co * cin + c) * 9 + tap];
          } else {
            const int tap = s / (cin / 32), c = 32 * (s % (cin / 32)) + k;
            wv = W[(co * cin + c) * 9 + tap];
          }
          uint16_t t[3];
          bx_split(wv, t[0], t[1], t[2]);
          for (int q = 0; q < 3; ++q) out[(((ot * nch + s) * 3 + q) * 64 + lane) * 8 + e] = t[q];
        }
}

// packed blob layout (floats): one entry per layer, fragments then the bias
struct ReprLayout {
  int w1, b1, r1w1, r1b1, r1w2, r1b2, dw, db1, dw2, db2, r2w1, r2b1, r2w2, r2b2, total;
};
inline int repr_frag_floats(int cout, int nch) { return cout / 16 * nch * 3 * 64 * 4; }
inline ReprLayout repr_layout() {
  ReprLayout L;
  int o = 0;
  auto take = [&](int n) { const int r = o; o += (n + 3) & ~3; return r; };
  L.w1 = take(repr_frag_floats(32, 2)); L.b1 = take(32);
  L.r1w1 = take(repr_frag_floats(32, 9)); L.r1b1 = take(32);
  L.r1w2 = take(repr_frag_floats(32, 9)); L.r1b2 = take(32);
  L.dw = take(repr_frag_floats(128, 9)); L.db1 = take(64);
  L.dw2 = take(repr_frag_floats(64, 18)); L.db2 = take(64);
  L.r2w1 = take(repr_frag_floats(64, 18)); L.r2b1 = take(64);
  L.r2w2 = take(repr_frag_floats(64, 18)); L.r2b2 = take(64);
  L.total = o;
  return L;
}

}  // namespace lzm
