// lzm_repr.h — the representation network's downsampling stages of the Atari configs (BASELINE.json configs 3
// and 5) on the split-fp16 matrix path: initial_inference's DownSample (lzero/model/common.py:164-265), with
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
// v_mfma_f32_16x16x32_f16 with every f32 operand split into two fp16 terms x = h + l (h = fp16(x), l =
// fp16(x - h): 22 significand bits, |x - h - l| <= 2^-22 |x|) and three products per K (w_h x_h, w_h x_l,
// w_l x_h; the dropped w_l x_l is below 2^-22 of |w x|): f32-level error at half the MFMAs of a three-term
// bf16 scheme. Range (lzm_conv.h's rule): out channel c's weight row is packed as W_c 2^e_c (its largest |w|
// in [2^14, 2^15)); a tile's input halo is split as x 2^s with s from the tile's exact max |x| (each wave's
// max of the values it splits meets the others' in LDS at one more barrier of the split pass); the epilogue
// multiplies by 2^-(e_c + s), exactly. ReLUs propagate NaN. A persistent grid (one 8-wave workgroup per CU)
// walks 64- or 128-pixel output tiles of whole image rows.
//
// Staging (the tile loop's memory side, no registers): a tile's input rows, and its residual, are contiguous in
// HBM (NHWC rows; the first layer: 9 rows of each NCHW plane), so they are copied as they lie into an LDS ring
// of raw f32 slots by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave-instruction), S = 2-3 tiles ahead of the
// MFMAs. Each tile then runs: counted vmcnt + barrier (the tile's slot has landed) -> split pass (raw f32 slot
// -> the two fp16 term images, halo borders zeroed) -> barrier -> DMA of tile n + S into the freed slot ->
// MFMAs -> epilogue (residual from its LDS slot). Only the DMA touches the VM counter inside the loop (the
// weights are waited for before it, the epilogue only stores), so every wait is an exact count of younger DMAs.
//
// LDS image of a halo, per fp16 term: [channel group g = 8 channels][position][8 fp16], a group's plane padded
// to a multiple of 16 positions. A B-fragment read (lane: pixel l & 15 of a 16-pixel tile, channel group
// g0 + (l >> 4)) touches 16 consecutive positions per group, so every ds_read_b128 lane group hits 16
// distinct 16-B bank slots. Stride-2 convolutions store the halo's even and odd columns apart, which makes
// their reads consecutive too. The first layer (C <= 7 input channels, NCHW) stages an im2col tile instead:
// K = tap * C + channel, zero-padded to 64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "lzm_conv.h"

namespace lzm {

constexpr int kRpThreads = 512;  // 8 waves: two per SIMD
constexpr int kRpTerms = 2;      // fp16 terms per f32 operand

typedef _Float16 rpf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ rpf16x8 rp_as(uint4 u) { return __builtin_bit_cast(rpf16x8, u); }

struct ReprConvArgs {
  int B, ntiles, cin_obs;  // cin_obs: first layer's input channels (MODE 2)
  const float *in;         // NHWC [B][HIN][HIN][CIN] (MODE 2: NCHW obs [B][cin_obs][64][64])
  const float *w;          // fragments [out tile][chunk][term][lane][8 fp16] (repr_pack)
  const float *winv;       // [COUT] 2^-e_c of the packed rows (MODE 1: 128, conv1's then the shortcut's)
  const float *bias;       // [COUT] (MODE 1: [64], the first half's)
  const float *res;        // NHWC residual of the output's shape (RES launches only)
  float *out;              // NHWC [B][HOUT][HOUT][COUT] (MODE 1: the first 64 channels)
  float *out2;             // MODE 1: the shortcut's 64 channels, NHWC
};

// Geometry of one layer: WOUT-wide output rows, 64-pixel tiles of TR rows; halo HR x HC (bordered), LDS row
// pitch ROWP (stride 2: even columns, then odd ones), group plane NPP positions (a multiple of 16).
template <int CIN, int COUT, int STRIDE, int WOUT, int MODE, bool RES>
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
  static constexpr int TERM = CG * NPP * 8;                           // fp16 per term image
  static constexpr int BUF = kRpTerms * TERM;                         // fp16 of the term images
  static constexpr int PPW = MODE == 2 ? 64 : 64 / CG;                // positions per wave-instruction
  // split items (position, group): 64 per wave-instruction, PPW consecutive positions x CG groups
  static constexpr int ITEMS = MODE == 2 ? PX * 8 : (HR * HC + PPW - 1) / PPW * 64;
  static constexpr int IPT = (ITEMS + kRpThreads - 1) / kRpThreads;  // per thread
  // raw DMA slot: MODE 2: [c < 7][RR = 2 TR + 1 rows][64] of the NCHW planes; else [HR][HIN][CIN] NHWC rows
  static constexpr int HIN = MODE == 2 ? 64 : WOUT * STRIDE;
  static constexpr int RR = 2 * TR + 1;
  static constexpr int RAW_F4 = MODE == 2 ? 7 * RR * 16 : HR * HIN * CIN / 4;  // float4 (MODE 2: for 7 planes)
  static constexpr int KRAW = (RAW_F4 + 511) / 512;                   // DMA wave-instructions per wave
  static constexpr int RAWB = KRAW * 8 * 1024;                        // bytes per raw slot
  static constexpr int COUT_T = MODE == 1 ? COUT / 2 : COUT;          // channels of one output tensor
  static constexpr int RES_F4 = RES ? PX * COUT_T / 4 : 0;            // the residual tile, as it lies
  static constexpr int KRES = (RES_F4 + 511) / 512;
  static constexpr int RESB = KRES * 8 * 1024;
  static constexpr int TERMB = BUF * 2;
  static constexpr int XSB = KS == 2 ? 8 * 64 * 8 * 4 : 0;            // K-split partial sums
  static constexpr int FIXB = 2 * RESB + XSB + 32;
  static constexpr int S = TERMB + 3 * RAWB + FIXB <= 160 * 1024 ? 3 : 2;  // raw ring depth
  static constexpr int RAW0 = TERMB, RES0 = RAW0 + S * RAWB, XS0 = RES0 + 2 * RESB;
  static constexpr int ZB = XS0 + XSB;  // 32 zero bytes: the split pass's source for halo positions off the image
  static constexpr int MX = ZB + 32;    // 8 words: the waves' maxima of a tile's halo (the split pass)
  static constexpr int LDSB = MX + 32;
  static_assert(LDSB <= 160 * 1024, "LDS");
  // a tile's wait at the top of its iteration: the DMAs younger than the newest copy it needs (the tile's raw
  // copy and residual): the raw copy issued with that residual (RES), or the S - 1 raw copies after it
  static constexpr int NTOP = RES ? KRAW : (S - 1) * KRAW;
  static_assert(NTOP < 64, "vmcnt");
};

// the LDS position of halo (row hr, bordered column hc)
template <class G, int STRIDE>
__device__ __forceinline__ int rp_pos(int hr, int hc) {
  if constexpr (STRIDE == 2) return hr * G::ROWP + (hc & 1) * G::HC2 + (hc >> 1);
  else return hr * G::ROWP + hc;
}

// split item q of a tile -> (LDS position, channel group); false past the last item
template <class G, int STRIDE, int MODE>
__device__ __forceinline__ bool rp_item(int q, int &hr, int &hc, int &g) {
  if (q >= G::ITEMS) return false;
  if constexpr (MODE == 2) {
    hr = 0;
    hc = q % G::PX;  // pixel of the tile
    g = q / G::PX;
    return true;
  }
  // lanes: PPW consecutive halo positions (distinct bank slots per 8-lane write group) x the CG channel groups
  const int lin = (q >> 6) * G::PPW + (q & 63) % G::PPW;
  if (lin >= G::HR * G::HC) return false;
  g = (q & 63) / G::PPW;
  hr = lin / G::HC;
  hc = lin % G::HC;
  return true;
}

// one LDS-DMA wave-instruction: 16 B from each lane's global address to lds_base + 16 lane (lds_base: a
// wave-uniform LDS byte address). Inline asm, so the compiler inserts no vmcnt waits of its own for it: the
// kernel counts its DMAs itself (rp_wait_vm)
__device__ __forceinline__ void rp_dma16(const void *gsrc, uint32_t lds_base) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_base)
               : "memory");
}

template <int N>
__device__ __forceinline__ void rp_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// every wave's LDS operations retired, then the workgroup barrier (no vmcnt: DMAs stay in flight across it)
__device__ __forceinline__ void rp_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// DMA of tile `tile`'s raw input rows into the raw slot at LDS byte address `slot` (tiles past the last one:
// the last tile again, so that every wave issues the same count). Rows outside the image load row 0 / HIN - 1
// (the split pass zeroes them)
template <int CIN, int COUT, int STRIDE, int WOUT, int MODE, bool RES>
__device__ __forceinline__ void rp_issue_raw(const ReprConvArgs &a, int tile, uint32_t slot, int wv, int lane) {
  typedef ReprGeom<CIN, COUT, STRIDE, WOUT, MODE, RES> G;
  constexpr int TPI = WOUT / G::TR;
  tile = min(tile, a.ntiles - 1);
  const int b = tile / TPI, r0 = (tile % TPI) * G::TR;
#pragma unroll
  for (int i = 0; i < G::KRAW; ++i) {
    const int f = (i * 8 + wv) * 64 + lane;
    const float *src;
    if constexpr (MODE == 2) {
      const int C = a.cin_obs, ff = min(f, C * G::RR * 16 - 1);
      const int c = ff / (G::RR * 16), rem = ff % (G::RR * 16);
      const int iy = min(max(2 * r0 - 1 + rem / 16, 0), 63);
      src = a.in + (((int64_t)b * C + c) * 64 + iy) * 64 + (rem % 16) * 4;
    } else {
      constexpr int ROWF4 = G::HIN * CIN / 4;
      const int ff = min(f, G::RAW_F4 - 1), hr = ff / ROWF4;
      const int iy = min(max(r0 * STRIDE - 1 + hr, 0), G::HIN - 1);
      src = a.in + ((int64_t)b * G::HIN + iy) * G::HIN * CIN + (ff % ROWF4) * 4;
    }
    rp_dma16(src, slot + (i * 8 + wv) * 1024);
  }
}

// DMA of tile `tile`'s residual (its output rows of a.res, as they lie) into the residual slot at `slot`
template <int CIN, int COUT, int STRIDE, int WOUT, int MODE, bool RES>
__device__ __forceinline__ void rp_issue_res(const ReprConvArgs &a, int tile, uint32_t slot, int wv, int lane) {
  typedef ReprGeom<CIN, COUT, STRIDE, WOUT, MODE, RES> G;
  constexpr int TPI = WOUT / G::TR;
  tile = min(tile, a.ntiles - 1);
  const int b = tile / TPI, r0 = (tile % TPI) * G::TR;
  const float *base = a.res + ((int64_t)b * WOUT + r0) * WOUT * G::COUT_T;
#pragma unroll
  for (int i = 0; i < G::KRES; ++i) {
    const int f = min((i * 8 + wv) * 64 + lane, G::RES_F4 - 1);
    rp_dma16(base + f * 4, slot + (i * 8 + wv) * 1024);
  }
}

// x = h + l: h = fp16(x), l = fp16(x - h) (x - h is exact in f32), both rounded to nearest, pairs packed
template <class F8>
__device__ __forceinline__ void rp_split8(const F8 &x, uint4 &h, uint4 &l) {
  typedef float f8 __attribute__((ext_vector_type(8)));
  const f8 xv = f8{x[0], x[1], x[2], x[3], x[4], x[5], x[6], x[7]};
  const rpf16x8 hv = __builtin_convertvector(xv, rpf16x8);
  const rpf16x8 lv = __builtin_convertvector(xv - __builtin_convertvector(hv, f8), rpf16x8);
  h = __builtin_bit_cast(uint4, hv);
  l = __builtin_bit_cast(uint4, lv);
}

// split pass: the tile's raw slot -> the two fp16 term images (halo borders and padding taps zero), scaled by
// 2^s from the halo's exact max (a barrier inside: every thread calls it); returns 2^-s
template <int CIN, int COUT, int STRIDE, int WOUT, int MODE, bool RES>
__device__ __forceinline__ float rp_split(const ReprConvArgs &a, const float *raw, const float *zero, uint16_t *buf,
                                          uint32_t *mslot, int r0, int wv, int lane) {
  typedef ReprGeom<CIN, COUT, STRIDE, WOUT, MODE, RES> G;
  typedef float f8 __attribute__((ext_vector_type(8)));
  f8 xs[G::IPT];
  int pos[G::IPT], grp[G::IPT];
  bool on[G::IPT];
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < G::IPT; ++i) {
    int hr, hc, g;
    on[i] = rp_item<G, STRIDE, MODE>(threadIdx.x + i * kRpThreads, hr, hc, g);
    grp[i] = g;
    f8 x = f8{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (on[i]) {
      if constexpr (MODE == 2) {
        // im2col: pixel hc of the tile (local row hc / WOUT, column hc % WOUT), K = 8 g + j = tap * C + c
        pos[i] = hc;
        const int C = a.cin_obs, lr = hc / WOUT, ox = hc % WOUT;
        int tap = (8 * g) / C, c = 8 * g - tap * C;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int rr = 2 * lr + tap / 3, ix = 2 * ox + tap % 3 - 1, iy = 2 * r0 - 1 + rr;
          const bool ok = tap < 9 && iy >= 0 && iy < 64 && ix >= 0 && ix < 64;
          const float v = raw[ok ? (c * G::RR + rr) * 64 + ix : 0];
          x[j] = __uint_as_float(__float_as_uint(v) & (ok ? 0xffffffffu : 0u));
          ++c;
          tap += c == C;
          c = c == C ? 0 : c;
        }
      } else {
        pos[i] = rp_pos<G, STRIDE>(hr, hc);
        const int iy = r0 * STRIDE - 1 + hr, ix = hc - 1;
        const bool ok = iy >= 0 && iy < G::HIN && ix >= 0 && ix < G::HIN;
        const float4 *src = reinterpret_cast<const float4 *>(ok ? raw + (hr * G::HIN + ix) * CIN + 8 * g : zero);
        const float4 u = src[0], v = src[1];
        x = f8{u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
      }
    }
    xs[i] = x;
#pragma unroll
    for (int j = 0; j < 8; ++j) m = max(m, __float_as_uint(x[j]) & 0x7fffffffu);
  }
  m = (uint32_t)xor_max((int)m);
  if (lane == 0) mslot[wv] = m;
  rp_barrier();
  const uint4 m0 = reinterpret_cast<const uint4 *>(mslot)[0], m1 = reinterpret_cast<const uint4 *>(mslot)[1];
  const uint32_t mm = max(max(max(m0.x, m0.y), max(m0.z, m0.w)), max(max(m1.x, m1.y), max(m1.z, m1.w)));
  const int s = bx_scale_exp(__uint_as_float(mm), kBxAExp);
  const float sc = bx_pow2(s);
#pragma unroll
  for (int i = 0; i < G::IPT; ++i) {
    if (!on[i]) continue;
    uint4 h, l;
    rp_split8(xs[i] * sc, h, l);
    const int o = (grp[i] * G::NPP + pos[i]) * 8;
    *reinterpret_cast<uint4 *>(buf + o) = h;
    *reinterpret_cast<uint4 *>(buf + G::TERM + o) = l;
  }
  return bx_pow2(-s);
}

template <int CIN, int COUT, int STRIDE, int WOUT, int MODE, bool RES>
__global__ __launch_bounds__(kRpThreads) __attribute__((amdgpu_waves_per_eu(2, 2))) void repr_conv_kernel(
    ReprConvArgs a) {
  typedef ReprGeom<CIN, COUT, STRIDE, WOUT, MODE, RES> G;
  extern __shared__ uint4 rp_lds4[];
  uint8_t *lb = reinterpret_cast<uint8_t *>(rp_lds4);
  uint16_t *terms = reinterpret_cast<uint16_t *>(lb);
  float *xscr = reinterpret_cast<float *>(lb + G::XS0);  // K-split partial sums
  const uint32_t lds0 = (uint32_t)reinterpret_cast<uintptr_t>(lb);  // the LDS byte address of the array
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  // this wave's out tile, first pixel tile and K half
  const int ot = G::OT == 2 ? (wv & 1) : (G::OT == 4 ? (wv & 3) : wv);
  const int pt0 = G::OT == 2 ? (wv >> 1) * G::PTW : 0;
  const int kh = G::KS == 2 ? (wv >> 2) : 0;
  // the weights of that out tile over its K chunks, both terms: registers for the whole launch
  uint4 wr[G::NCW][kRpTerms];
#pragma unroll
  for (int s = 0; s < G::NCW; ++s)
#pragma unroll
    for (int q = 0; q < kRpTerms; ++q)
      wr[s][q] = reinterpret_cast<const uint4 *>(a.w)[((ot * G::NCH + kh * G::NCW + s) * kRpTerms + q) * 64 + lane];
  // out channels 4 (lane >> 4) .. + 3 of the tile; the dual layer's upper half is the shortcut (no bias)
  constexpr int COUT_T = G::COUT_T;
  constexpr int HOUT = WOUT, TPI = HOUT / G::TR;
  int ch = 16 * ot + 4 * (lane >> 4);
  const bool sc = MODE == 1 && ch >= COUT_T;
  float *dst = sc ? a.out2 : a.out;
  if (sc) ch -= COUT_T;
  const float4 bias = sc ? float4{0.f, 0.f, 0.f, 0.f} : *reinterpret_cast<const float4 *>(a.bias + ch);
  const float4 wsc = *reinterpret_cast<const float4 *>(a.winv + 16 * ot + 4 * (lane >> 4));  // the packed rows' 2^-e
  // the compiler's own loads retired here (a builtin wait it accounts for): inside the loop the VM counter
  // holds DMAs and stores only
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
  if (tid < 8) reinterpret_cast<float *>(lb + G::ZB)[tid] = 0.f;  // (ordered by the first tile's barrier)
  const int grid = gridDim.x;
  int tile = blockIdx.x;
  // prologue: raw copies of tiles 0 .. S - 1 (the residual of tile 0 before the last one: the order the
  // loop's waits count)
#pragma unroll
  for (int k = 0; k < G::S - 1; ++k)
    rp_issue_raw<CIN, COUT, STRIDE, WOUT, MODE, RES>(a, tile + k * grid, lds0 + G::RAW0 + k * G::RAWB, wv, lane);
  if constexpr (RES) rp_issue_res<CIN, COUT, STRIDE, WOUT, MODE, RES>(a, tile, lds0 + G::RES0, wv, lane);
  rp_issue_raw<CIN, COUT, STRIDE, WOUT, MODE, RES>(a, tile + (G::S - 1) * grid,
                                                    lds0 + G::RAW0 + (G::S - 1) * G::RAWB, wv, lane);
  const float *zero = reinterpret_cast<const float *>(lb + G::ZB);
  int slot = 0;  // the raw slot of the current tile (n mod S)
  for (int it = 0; tile < a.ntiles; ++it, tile += grid) {
    const int b = tile / TPI, r0 = (tile % TPI) * G::TR;
    rp_wait_vm<G::NTOP>();  // this wave's copies landed ...
    rp_barrier();           // ... and every wave's; every wave is also done with the previous tile's LDS
    const float rinv = rp_split<CIN, COUT, STRIDE, WOUT, MODE, RES>(
        a, reinterpret_cast<const float *>(lb + G::RAW0 + slot * G::RAWB), zero, terms,
        reinterpret_cast<uint32_t *>(lb + G::MX), r0, wv, lane);
    rp_barrier();
    // refill: the next tile's residual into the other residual slot, tile n + S into the slot of tile n
    if constexpr (RES)
      rp_issue_res<CIN, COUT, STRIDE, WOUT, MODE, RES>(a, tile + grid, lds0 + G::RES0 + ((it + 1) & 1) * G::RESB,
                                                        wv, lane);
    rp_issue_raw<CIN, COUT, STRIDE, WOUT, MODE, RES>(a, tile + G::S * grid, lds0 + G::RAW0 + slot * G::RAWB, wv,
                                                      lane);
    slot = slot + 1 == G::S ? 0 : slot + 1;
    bxf4 acc[G::PTW];
#pragma unroll
    for (int p = 0; p < G::PTW; ++p) acc[p] = bxf4{0.f, 0.f, 0.f, 0.f};
    // B fragments of chunk s for the wave's pixel tiles (lane: pixel 16 (pt0 + p) + (lane & 15) of the tile,
    // output row px / WOUT, column px % WOUT; channel group 4 j + (lane >> 4))
    auto load_x = [&](int s, uint4 (&x)[G::PTW][kRpTerms]) {
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
        for (int q = 0; q < kRpTerms; ++q)
          x[p][q] = *reinterpret_cast<const uint4 *>(terms + q * G::TERM + (g * G::NPP + pos) * 8);
      }
    };
    // software pipeline: chunk s + 1's LDS reads issued before chunk s's MFMAs (the scheduling barrier keeps
    // the compiler from hoisting every chunk's reads to the top, which would need 9 x the fragment registers)
    uint4 xa[G::PTW][kRpTerms], xb[G::PTW][kRpTerms];
    load_x(0, xa);
#pragma unroll
    for (int s = 0; s < G::NCW; ++s) {
      uint4(&xc)[G::PTW][kRpTerms] = (s & 1) ? xb : xa;
      uint4(&xn)[G::PTW][kRpTerms] = (s & 1) ? xa : xb;
      if (s + 1 < G::NCW) load_x(s + 1, xn);
      const uint4(&w)[kRpTerms] = wr[s];
#pragma unroll
      for (int p = 0; p < G::PTW; ++p) {
        // small terms first: w_l x_h, w_h x_l, w_h x_h
        bxf4 c = acc[p];
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(rp_as(w[1]), rp_as(xc[p][0]), c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(rp_as(w[0]), rp_as(xc[p][1]), c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(rp_as(w[0]), rp_as(xc[p][0]), c, 0, 0, 0);
        acc[p] = c;
      }
      // the order within the chunk (left alone, the scheduler sinks chunk s + 1's fragment reads to the end of
      // chunk s and every chunk then waits out a full LDS latency): two pixel tiles, the reads first, then the
      // MFMAs; four (64-channel layers, 64 fragment registers), half the reads after the first tile's MFMAs and
      // half after the third's, within the register file
      if constexpr (G::PTW == 2) {
        if (s + 1 < G::NCW) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);  // DS reads
        __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);                       // MFMAs
      } else if (s + 1 < G::NCW) {
        __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 6, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
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
      rp_barrier();
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
    // epilogue: acc[p][r] = out channel ch + r at pixel 16 (pt0 + p) + (lane & 15), scaled by 2^(e + s)
    const float *rs = reinterpret_cast<const float *>(lb + G::RES0 + (it & 1) * G::RESB);
    const float4 f = float4{wsc.x * rinv, wsc.y * rinv, wsc.z * rinv, wsc.w * rinv};
#pragma unroll
    for (int p = 0; p < G::PTW; ++p) {
      if (G::KS == 2 && (p >> 1) != kh) continue;  // (the K-split partner's tiles)
      const int px = 16 * (pt0 + p) + (lane & 15);
      const int64_t e = (((int64_t)b * HOUT + r0 + px / WOUT) * WOUT + px % WOUT) * COUT_T + ch;
      float4 y = float4{__fmaf_rn(acc[p][0], f.x, bias.x), __fmaf_rn(acc[p][1], f.y, bias.y),
                        __fmaf_rn(acc[p][2], f.z, bias.z), __fmaf_rn(acc[p][3], f.w, bias.w)};
      if (!sc) {
        if constexpr (RES) {
          const float4 rr = *reinterpret_cast<const float4 *>(rs + px * COUT_T + ch);
          y.x += rr.x; y.y += rr.y; y.z += rr.z; y.w += rr.w;
        }
        // relu, NaN kept (torch's)
        y.x = y.x < 0.f ? 0.f : y.x; y.y = y.y < 0.f ? 0.f : y.y; y.z = y.z < 0.f ? 0.f : y.z; y.w = y.w < 0.f ? 0.f : y.w;
      }
      *reinterpret_cast<float4 *>(dst + e) = y;
    }
  }
  rp_wait_vm<0>();  // the copies of tiles past the end land before the workgroup's LDS is released
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
// A-operand fragments of one convolution: W [cout][cin][3][3] (folded), each row c scaled by 2^e_c (inv[c] =
// 2^-e_c) -> [out tile][chunk][term][lane][8 fp16], lane -> out channel 16 tile + (lane & 15), K = 8 (lane >> 4)
// + e within the chunk; chunk s = tap * (cin / 32) + j with K -> in channel 32 j + ..., or (first layer, cin <= 7)
// chunk s with K = 32 s + ... = tap * cin + c. Two weights stacked (the dual layer: W [64] then W3 [64]) give
// cout = 128.
inline void repr_pack(const float *W, int cout, int cin, bool im2col, float *outf, float *inv) {
  uint16_t *out = reinterpret_cast<uint16_t *>(outf);
  const int nch = im2col ? 2 : 9 * (cin / 32);
  std::vector<int> er(cout);
  for (int co = 0; co < cout; ++co) {
    double l1;
    er[co] = bx_row_exp(W + (size_t)co * cin * 9, cin * 9, &l1);
    inv[co] = bx_pow2(-er[co]);
  }
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
          wv = ldexpf(wv, er[co]);
          const _Float16 h = (_Float16)wv, l = (_Float16)(wv - (float)h);  // the kernel's split, rp_split8
          const uint16_t t[kRpTerms] = {__builtin_bit_cast(uint16_t, h), __builtin_bit_cast(uint16_t, l)};
          for (int q = 0; q < kRpTerms; ++q) out[(((ot * nch + s) * kRpTerms + q) * 64 + lane) * 8 + e] = t[q];
        }
}

// packed blob layout (floats): one entry per layer, fragments then the bias
struct ReprLayout {
  int w1, b1, r1w1, r1b1, r1w2, r1b2, dw, db1, dw2, db2, r2w1, r2b1, r2w2, r2b2;
  int s1, r1s1, r1s2, ds, ds2, r2s1, r2s2;  // the layers' row scales 2^-e_c (ds: 128, the dual layer's)
  int total;
};
inline int repr_frag_floats(int cout, int nch) { return cout / 16 * nch * kRpTerms * 64 * 4; }
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
  L.s1 = take(32); L.r1s1 = take(32); L.r1s2 = take(32); L.ds = take(128); L.ds2 = take(64); L.r2s1 = take(64);
  L.r2s2 = take(64);
  L.total = o;
  return L;
}

}  // namespace lzm
