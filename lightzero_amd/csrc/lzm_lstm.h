// lzm_lstm.h — the EfficientZero reward LSTM of the recurrent step around one batched gate GEMM
// (config 3, Pong EZ).
//
// Per simulation the reference (mcts_ctree.py:756-816, efficientzero_model.py:526-574) gathers the
// leaf's (h, c) LSTM state from the per-simulation state lists, runs one nn.LSTM step on the
// flattened reward planes, and after the network zeroes the new state of every root whose
// search_len % lstm_horizon_len == 0 before appending it to the lists. As PyTorch ops that is two
// gathers, a concat, the gate GEMM, nine pointwise launches and three more for the reset mask. Here:
//   ez_lstm_input_kernel  xin[b] = [r[b] | hpool[x[b]][b]]              (gather + concat)
//   gates = xin @ W^T + bias                                           (plain GEMM: rocBLAS)
//   ez_lstm_cell_kernel   i, f, g, o = gates chunks (nn.LSTM order); c1 = s(f) c0 + s(i) tanh(g);
//                         h1 = s(o) tanh(c1) with c0 = cpool[x[b]][b]; h1 / c1 out unmasked (the
//                         value-prefix head reads h1), and masked into the next state slot
//                         (zero where search_len % horizon == 0, mcts_ctree.py:810-813).
// Both are float4-vectorised grid-stride passes: HBM/L2 bound, ~3 MB per simulation at B = 256.
// ez_lstm_gemm_cell_kernel (below) replaces the GEMM and the cell pass with one launch.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <vector>

#include "lzm_conv.h"

namespace lzm {

__global__ __launch_bounds__(256) void ez_lstm_input_kernel(int B, int Kr, int H, const float *r, const float *hpool,
                                                            const int32_t *x, float *xin) {
  const int K4 = (Kr + H) >> 2, Kr4 = Kr >> 2, H4 = H >> 2;
  const long long n = (long long)B * K4;
  for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < n; q += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(q / K4), k = (int)(q - (long long)b * K4);
    float4 v;
    if (k < Kr4)
      v = reinterpret_cast<const float4 *>(r)[(size_t)b * Kr4 + k];
    else
      v = reinterpret_cast<const float4 *>(hpool)[((size_t)max(x[b], 0) * B + b) * H4 + (k - Kr4)];
    reinterpret_cast<float4 *>(xin)[q] = v;
  }
}

__device__ inline float lstm_sigmoid(float v) { return 1.0f / (1.0f + expf(-v)); }

__global__ __launch_bounds__(256) void ez_lstm_cell_kernel(int B, int H, const float *gates, const float *cpool,
                                                           const int32_t *x, const int32_t *search_len, int horizon,
                                                           float *h1, float *c1, float *hslot, float *cslot) {
  const int H4 = H >> 2;
  const long long n = (long long)B * H4;
  for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < n; q += (long long)gridDim.x * blockDim.x) {
    const int b = (int)(q / H4), j = (int)(q - (long long)b * H4);
    const float4 *g4 = reinterpret_cast<const float4 *>(gates) + (size_t)b * 4 * H4;
    const float4 gi = g4[j], gf = g4[H4 + j], gg = g4[2 * H4 + j], go = g4[3 * H4 + j];
    const float4 c0 = reinterpret_cast<const float4 *>(cpool)[((size_t)max(x[b], 0) * B + b) * H4 + j];
    float4 c, h;
#define LZM_LSTM_LANE(m)                                                          \
  c.m = lstm_sigmoid(gf.m) * c0.m + lstm_sigmoid(gi.m) * tanhf(gg.m);             \
  h.m = lstm_sigmoid(go.m) * tanhf(c.m);
    LZM_LSTM_LANE(x)
    LZM_LSTM_LANE(y)
    LZM_LSTM_LANE(z)
    LZM_LSTM_LANE(w)
#undef LZM_LSTM_LANE
    reinterpret_cast<float4 *>(h1)[q] = h;
    reinterpret_cast<float4 *>(c1)[q] = c;
    const bool reset = horizon > 0 && (search_len[b] % horizon) == 0;
    const float4 z = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    reinterpret_cast<float4 *>(hslot)[q] = reset ? z : h;
    reinterpret_cast<float4 *>(cslot)[q] = reset ? z : c;
  }
}

// ---- the gate GEMM and the cell in one launch, on split-fp16 MFMA (lzm_conv.h's split scheme)
//
// gates = xin W^T + b is M = B rows x N = 4H columns x K; rocBLAS ran it in f32 (16 us at Pong's
// 256 x 2048 x 1536) and the cell was a second pass over the gates in HBM. Here a tile is 64 rows
// (envs) x 16 hidden units, i.e. the 64 gate columns {i, f, g, o} x 16 units, so the cell runs in the
// GEMM's epilogue from registers. Operands: each f32 value is held as h + l (two fp16 terms, an exact
// split: 22 significand bits) and every product is summed from the three terms l.h, h.l, h.h
// (v_mfma_f32_16x16x32_f16), as in the conv trunk.
// Range (lzm_conv.h): W's row (gate column) j is packed as W_j 2^e_j (its largest |w| in [2^14, 2^15)) and
// xin row b is split as x 2^s_b with s_b = 14 - floor(log2 max(M_r, 1)), M_r the exact max of the row's reward
// planes (|h| < 1): the trunk that writes the row computes it (xscale[b], or the EZ search's hand-off flag);
// the epilogue multiplies by 2^-(e_j + s_b), exactly. Every split value is checked (|x 2^s| < 65504, finite)
// into the range error word.
//   * 512 threads, two waves per SIMD: wave w owns column tile w & 3 (units 4 (w & 3) .. + 3, column
//     4 u + gate) and row half w >> 2 (two 16-row tiles). The four gates of a (row, unit) then sit in
//     the four lanes of a quad, and one DPP broadcast per gate hands them to the lane that writes it.
//   * Split K in two: the tile's two K halves run in two workgroups; the upper half (lower block ids,
//     dispatched first, so its partner is always resident) leaves its partial sums in a workspace and
//     raises a flag, the lower half adds them (lower + upper) and runs the cell. 256 workgroups at
//     B = 256 (every CU), 126 MB of L2 reads instead of 201 MB for 64 x 32 tiles without the split.
//   * Per 64-K stage both operands go through LDS, double-buffered, one barrier per stage: xin rows
//     are loaded as f32 and split on the fly ([term][row][64 K] fp16, 16-B chunk c of row r at
//     c ^ (r & 7), then 64 row scales); W comes pre-split from the host in MFMA fragment order
//     ([n-block][column tile][32-K chunk][term][lane][8 fp16], copied as is). Global loads run two
//     stages ahead.
//   * Tiles are mapped XCD by XCD (block id % 8 = XCD), whole n-blocks per XCD, so an XCD's L2 holds
//     its slice of W and every row of xin.
constexpr int kLsRows = 64;                      // rows (envs) per tile
constexpr int kLsUnits = 16;                     // hidden units per tile (64 gate columns)
constexpr int kLsKc = 64;                        // K per LDS stage
constexpr int kLsThreads = 512;
constexpr int kLsTerms = 2;                      // fp16 terms per f32 operand
constexpr int kLsPlane = kLsRows * kLsKc;        // 16-bit elements per A term plane
constexpr int kLsABuf = kLsTerms * kLsPlane;     // A stage (the term planes)
constexpr int kLsBBuf = 2 * 4 * kLsTerms * 64 * 8;  // B stage [chunk 2][col tile 4][term][lane][8]
constexpr int kLsStage = kLsABuf + kLsBBuf;      // 16-bit elements per stage buffer
constexpr int kLsLdsBytes = 2 * kLsStage * 2;    // two stage buffers
constexpr int kLsPartFloats = kLsThreads * 8;    // one tile's partial sums (8 per thread)

struct LstmArgs {
  int B, K, H, nmb, splitk;  // nmb = ceil(B / 64); splitk 1 or 2
  const float *xin;          // [B][K]
  const int32_t *xscale;     // [B] the rows' scale exponents s_b (lzm_conv_trunk_xin_p)
  int32_t *range_err;        // nullable: split values out of range (sticky)
  const uint4 *wf;           // fragments (lzm_ez_lstm_prepare)
  const float *winv;         // [4H] 2^-e_j of gate column j (lzm_ez_lstm_prepare, after the fragments)
  const float *bias;         // [4H] (b_ih + b_hh), nn.LSTM gate order
  const float *cpool;        // [slots][B][H]
  const int32_t *x, *search_len;
  int horizon;
  float *h1, *c1, *hslot, *cslot;  // [B][H]
  float *part;                     // split K: [tiles][kLsPartFloats]
  uint32_t *flags;                 // split K: [tiles], 0 between launches
  int32_t *err;                    // split K: bounded-spin timeouts (sticky)
  unsigned long long *stamps;      // diagnostics (nullptr in production): [block][8] 100 MHz real-time stamps
};

inline int64_t ls_frag_floats(int K, int H) { return (int64_t)K * 4 * H * kLsTerms / 2; }

// fragment element (nb, column tile, chunk, term, lane, e) <- W[(gate H + unit) K + k] 2^e_(gate H + unit);
// then the 4H inverse column scales
inline void ls_pack(const float *W, int K, int H, float *outf) {
  uint16_t *out = reinterpret_cast<uint16_t *>(outf);
  float *winv = outf + ls_frag_floats(K, H);
  const int nch = K / 32, NB = H / kLsUnits;
  std::vector<int> e((size_t)4 * H);
  for (int j = 0; j < 4 * H; ++j) {
    double l1;
    e[j] = bx_row_exp(W + (size_t)j * K, K, &l1);
    winv[j] = bx_pow2(-e[j]);
  }
  for (int nb = 0; nb < NB; ++nb)
    for (int w = 0; w < 4; ++w)
      for (int j = 0; j < nch; ++j)
        for (int lane = 0; lane < 64; ++lane)
          for (int el = 0; el < 8; ++el) {
            const int n = lane & 15, unit = kLsUnits * nb + 4 * w + (n >> 2), gate = n & 3;
            const int k = 32 * j + 8 * (lane >> 4) + el;
            const size_t row = (size_t)gate * H + unit;
            uint16_t t[kLsTerms];
            bx_split2(ldexpf(W[row * K + k], e[row]), t[0], t[1]);
            for (int q = 0; q < kLsTerms; ++q)
              out[((((size_t)(nb * 4 + w) * nch + j) * kLsTerms + q) * 64 + lane) * 8 + el] = t[q];
          }
}

__device__ __forceinline__ float ls_quad_bcast(float v, int g) {
  const int x = __builtin_bit_cast(int, v);
  const int r = g == 0 ? __builtin_amdgcn_update_dpp(0, x, 0x00, 0xF, 0xF, false)
              : g == 1 ? __builtin_amdgcn_update_dpp(0, x, 0x55, 0xF, 0xF, false)
              : g == 2 ? __builtin_amdgcn_update_dpp(0, x, 0xAA, 0xF, 0xF, false)
                       : __builtin_amdgcn_update_dpp(0, x, 0xFF, 0xF, 0xF, false);
  return __builtin_bit_cast(float, r);
}

// The split pass of N stage values of one row scaled by sc = 2^s_b: the two term vectors (pairs packed). (A row
// whose scale is clamped, s_b = -kBxAExp — reward planes beyond ~2^114 or not finite — counts as a range error
// where the scales are read: ls_row_bad.)
typedef float ls_f2 __attribute__((ext_vector_type(2)));
typedef _Float16 ls_h2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int ls_row_bad(int s) { return s <= -kBxAExp; }
template <int N>
__device__ __forceinline__ void ls_split_row(const float (&v)[N], float sc, uint32_t (&hh)[N / 2], uint32_t (&ll)[N / 2]) {
#pragma unroll
  for (int j = 0; j < N / 2; ++j) {
    const ls_f2 pr = ls_f2{v[2 * j], v[2 * j + 1]} * sc;
    const ls_h2 th = __builtin_convertvector(pr, ls_h2);
    const ls_h2 tq = __builtin_convertvector(pr - __builtin_convertvector(th, ls_f2), ls_h2);
    hh[j] = __builtin_bit_cast(uint32_t, th);
    ll[j] = __builtin_bit_cast(uint32_t, tq);
  }
}

__global__ __launch_bounds__(kLsThreads) void ez_lstm_gemm_cell_kernel(LstmArgs p) {
  extern __shared__ uint4 ls_lds4[];
  uint16_t *lds = reinterpret_cast<uint16_t *>(ls_lds4);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, ct = wv & 3, mh = wv >> 2;
  const int NB = p.H / kLsUnits, T = NB * p.nmb;
  // block -> (K half, tile): the upper K half takes the lower block ids; tiles XCD-major
  const int kh = p.splitk == 2 && (int)blockIdx.x < T ? 1 : 0;
  int q = (int)blockIdx.x - (p.splitk == 2 && kh == 0 ? T : 0);
  if ((T & 7) == 0) q = (q & 7) * (T >> 3) + (q >> 3);
  const int nb = q / p.nmb, mb = q - nb * p.nmb;
  const int row0 = kLsRows * mb, B = p.B, K = p.K, H = p.H;
  const int nch = K / 32, kspan = K / p.splitk, nst = kspan / kLsKc, k0 = kh * kspan;
  const int gate = lane & 3, unit = kLsUnits * nb + 4 * ct + ((lane & 15) >> 2);
  auto stamp = [&](int i) {
    if (p.stamps && tid == 0) p.stamps[blockIdx.x * 8 + i] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  // ---- staging: thread -> A (row tid / 8, 8 K values at 8 (tid % 8)) and 2 B uint4s per stage
  const int sr = tid >> 3, sseg = tid & 7;
  const bool srow = row0 + sr < B;
  const int sexp = srow ? p.xscale[row0 + sr] : 0;
  const float ssc = bx_pow2(sexp);  // the staged row's scale
  const int bad = sseg == 0 && ls_row_bad(sexp);
  const float4 *asrc = reinterpret_cast<const float4 *>(p.xin + (size_t)(srow ? row0 + sr : 0) * K + k0) + 2 * sseg;
  const uint4 *bsrc = p.wf + (size_t)nb * 4 * nch * kLsTerms * 64;  // [col tile][chunk][term][lane]
  // staging registers of two stages (native vector types: HIP's uint4 / float4 structs kept these
  // arrays in scratch)
  typedef unsigned ls_u4 __attribute__((ext_vector_type(4)));
  typedef float ls_f4 __attribute__((ext_vector_type(4)));
  ls_f4 va0[2], va1[2];
  ls_u4 vb0[kLsTerms], vb1[kLsTerms];
  const ls_u4 *bsrc4 = reinterpret_cast<const ls_u4 *>(bsrc);
  const ls_f4 *asrc4 = reinterpret_cast<const ls_f4 *>(asrc);
  // B stage = [chunk c][col tile][term][lane]: element e = tid + 512 u of 2 x 4 x kLsTerms x 64 uint4s
  constexpr int kBc = 4 * kLsTerms * 64, kBt = kLsTerms * 64;  // uint4s per chunk, per column tile
  static_assert(2 * kBc == kLsTerms * kLsThreads, "B stage: kLsTerms uint4s per thread");
  auto load_stage = [&](int s, ls_f4(&VA)[2], ls_u4(&VB)[kLsTerms]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 2; ++u) VA[u] = srow ? asrc4[s * (kLsKc / 4) + u] : ls_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < kLsTerms; ++u) {
      const int e = tid + kLsThreads * u, c = e / kBc, r = e - c * kBc, tl = r / kBt, rest = r - tl * kBt;
      const int j = (k0 / 32) + 2 * s + c;
      VB[u] = bsrc4[((size_t)tl * nch + j) * kBt + rest];
    }
  };
  auto store_stage = [&](int bsel, const ls_f4(&VA)[2], const ls_u4(&VB)[kLsTerms]) __attribute__((always_inline)) {
    const float v[8] = {VA[0][0], VA[0][1], VA[0][2], VA[0][3], VA[1][0], VA[1][1], VA[1][2], VA[1][3]};
    uint32_t h[4], l[4];
    ls_split_row<8>(v, ssc, h, l);
    uint16_t *abuf = lds + bsel * kLsStage;
    uint16_t *base = abuf + sr * kLsKc + ((sseg ^ (sr & 7)) & 7) * 8;
    *reinterpret_cast<uint4 *>(base) = uint4{h[0], h[1], h[2], h[3]};
    *reinterpret_cast<uint4 *>(base + kLsPlane) = uint4{l[0], l[1], l[2], l[3]};
    ls_u4 *bbuf = reinterpret_cast<ls_u4 *>(abuf + kLsABuf);
#pragma unroll
    for (int u = 0; u < kLsTerms; ++u) bbuf[tid + kLsThreads * u] = VB[u];
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  load_stage(0, va0, vb0);
  if (nst > 1) load_stage(1, va1, vb1);
  store_stage(0, va0, vb0);
  stamp(1);
  bxf4 acc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) acc[t] = bxf4{0.f, 0.f, 0.f, 0.f};
  const int ar = lane & 15, ag = lane >> 4;
  auto stage = [&](int s, auto par) __attribute__((always_inline)) {
    constexpr int PAR = decltype(par)::value;
    __syncthreads();
    if (s + 2 < nst) {
      if constexpr (PAR == 0)
        load_stage(s + 2, va0, vb0);
      else
        load_stage(s + 2, va1, vb1);
    }  // (slot PAR went to LDS at the end of stage s - 1)
    const uint16_t *abuf = lds + PAR * kLsStage;
    const uint4 *bbuf = reinterpret_cast<const uint4 *>(abuf + kLsABuf);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      uint4 a[2][kLsTerms], w[kLsTerms];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int r = 32 * mh + 16 * t + ar, o = r * kLsKc + (((4 * c + ag) ^ (r & 7)) & 7) * 8;
#pragma unroll
        for (int tm = 0; tm < kLsTerms; ++tm) a[t][tm] = *reinterpret_cast<const uint4 *>(abuf + tm * kLsPlane + o);
      }
#pragma unroll
      for (int tm = 0; tm < kLsTerms; ++tm) w[tm] = bbuf[((c * 4 + ct) * kLsTerms + tm) * 64 + lane];
      // small terms first: l.h, h.l, h.h (the conv trunk's order)
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bx_ash(a[t][1]), bx_ash(w[0]), acc[t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bx_ash(a[t][0]), bx_ash(w[1]), acc[t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bx_ash(a[t][0]), bx_ash(w[0]), acc[t], 0, 0, 0);
    }
    if (s + 1 < nst) {
      if constexpr (PAR == 0)
        store_stage(1, va1, vb1);
      else
        store_stage(0, va0, vb0);
    }
  };
  for (int s = 0; s < nst; s += 2) {
    stage(s, I0());
    if (s + 1 < nst) stage(s + 1, I1());
  }
  stamp(2);
  if (bad && p.range_err) atomicAdd(p.range_err, 1);
  // the cell's inputs for this lane's rows (lower K half only): issued after the GEMM's loads (vmcnt
  // counts in order: issued first, the dependent x -> cpool gather would hold up the first stage),
  // in flight during the hand-off
  float c0[2] = {0.f, 0.f}, bias_l = 0.f, wsc = 0.f, rsc[2][4] = {};
  int rst[2] = {0, 0};
  if (kh == 0) {
    bias_l = p.bias[(size_t)gate * H + unit];
    wsc = p.winv[(size_t)gate * H + unit];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int b = row0 + 32 * mh + 16 * t + 4 * (lane >> 4) + gate;
      if (b < B) {
        c0[t] = p.cpool[((size_t)max(p.x[b], 0) * B + b) * H + unit];
        rst[t] = p.horizon > 0 && (p.search_len[b] % p.horizon) == 0;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // accumulator row 32 mh + 16 t + 4 (lane >> 4) + r: 2^-(e_j + s_row)
        const int br = row0 + 32 * mh + 16 * t + 4 * (lane >> 4) + r;
        rsc[t][r] = wsc * (br < B ? bx_pow2(-p.xscale[br]) : 1.f);
      }
    }
  }
  // ---- split K: the upper half hands its partial sums over; the lower half adds them. Hand-off
  // (MI355X_MICROARCH.md, cross-CU hand-off table, first row): payload and flag stored sc1 (16-B buffer
  // stores with the sc1 policy; the flag by an agent-scope relaxed atomic), every storing wave's
  // vmcnt(0) and a workgroup barrier before the one flag store; the consumer's one lane polls the flag
  // sc1, a barrier, then sc1 payload loads.
  if (p.splitk == 2) {
    // payload: 16-B buffer stores / loads with the sc1 cache policy (aux = 16)
    typedef unsigned ls_u4v __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(p.part + (size_t)q * kLsPartFloats, 0, kLsPartFloats * 4, 0x00020000);
    if (kh == 1) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(ls_u4v, acc[t]), rs, (tid * 8 + 4 * t) * 4, 0, 16);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) __hip_atomic_store(p.flags + q, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      stamp(3);
      return;
    }
    if (tid == 0) {
      long long spins = 0;
      while (__hip_atomic_load(p.flags + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) {
        if (++spins > (1ll << 24)) {
          atomicAdd(p.err, 1);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      __hip_atomic_store(p.flags + q, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    stamp(3);
#pragma unroll
    for (int t = 0; t < 2; ++t)
      acc[t] += __builtin_bit_cast(bxf4, __builtin_amdgcn_raw_buffer_load_b128(rs, (tid * 8 + 4 * t) * 4, 0, 16));
  }
  // ---- epilogue: the column's weight scale undone, + bias, the four gates of (row, unit) from the quad, the
  // cell by lane gate = r (ez_lstm_cell_kernel's operations in its order)
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    float gi = 0.f, gf = 0.f, gg = 0.f, go = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = __fmaf_rn(acc[t][r], rsc[t][r], bias_l);
      const float vi = ls_quad_bcast(v, 0), vf = ls_quad_bcast(v, 1), vg = ls_quad_bcast(v, 2), vo = ls_quad_bcast(v, 3);
      if (gate == r) { gi = vi; gf = vf; gg = vg; go = vo; }
    }
    const int b = row0 + 32 * mh + 16 * t + 4 * (lane >> 4) + gate;
    if (b < B) {
      const float c = lstm_sigmoid(gf) * c0[t] + lstm_sigmoid(gi) * tanhf(gg);
      const float h = lstm_sigmoid(go) * tanhf(c);
      const size_t o = (size_t)b * H + unit;
      p.h1[o] = h;
      p.c1[o] = c;
      p.hslot[o] = rst[t] ? 0.0f : h;
      p.cslot[o] = rst[t] ? 0.0f : c;
    }
  }
  stamp(4);
}

// ---- one gate-GEMM + cell tile inside a persistent launch (the EfficientZero one-launch search,
// lzm_search_conv.h): 256 threads, same tile (64 rows x 16 hidden units, K split in two halves over
// two workgroups), same operand layouts, stage pipeline, scales and MFMA order as ez_lstm_gemm_cell_kernel,
// so every output bit is the same. Wave w owns column tile w and all four 16-row tiles (the 512-thread
// kernel gives each wave two); the staging thread map changes with the thread count (thread -> row
// 16 w + 4 u + lane / 16, 4 values), the LDS layout does not. The xin rows are read with sc1 loads (they were
// handed over by other workgroups, MI355X_MICROARCH.md's first hand-off row).
typedef unsigned lp_u4 __attribute__((ext_vector_type(4)));
typedef float lp_f4 __attribute__((ext_vector_type(4)));
constexpr int kLpThreads = 256;
#ifndef LZM_LP_DEPTH
#define LZM_LP_DEPTH 2  // register sets of staged loads: global loads run LZM_LP_DEPTH - 1 stages ahead (2..4)
#endif

struct LpTile {
  int row0, nb, kh;  // tile rows [row0, row0 + 64), hidden units [16 nb, 16 nb + 16), K half
};

// the GEMM part: acc[t] = the tile's K-half partial sums (row tile t = rows 16 t .. + 15 of the tile,
// this wave's 16 gate columns; still scaled by 2^(e_j + s_row)), accumulated exactly as the 512-thread
// kernel does. rexp: the tile's 64 row scale exponents (LDS); bad: |= a split value out of range.
// lds: kLsLdsBytes of staging; xr: buffer resource over xin [B][K] (num_records = B * K * 4);
// wfrag: ls_pack's split-fp16 fragments (lzm_ez_lstm_prepare, the ones ez_lstm_gemm_cell_kernel reads). A
// is read as f32 and split on the fly (a thread stages 4 values of 4 rows through LDS); a wave loads
// the B fragments its own MFMAs consume (chunk 0 and 1, column tile = the wave, its lane, both terms)
// straight into registers: B never touches LDS. (Measured: B read as f32 in the same order and split
// on the device — two thirds of the bytes — made the GEMM slower, 29 K -> 33 K cycles per
// simulation: the split's VALU work sits on the stage's critical path, the bytes do not.)
// Loads go through buffer resources (one 32-bit per-thread offset each, the stage in the scalar
// offset): no 64-bit address per load for the compiler to hoist out of the simulation loop and spill.
__device__ __forceinline__ void lp_tile_gemm(const LpTile &tl, int B, int K, const __amdgpu_buffer_rsrc_t xr,
                                             const uint16_t *wfrag, const int *rexp, uint16_t *lds, bxf4 (&acc)[4],
                                             int &bad) {
  const int tid = threadIdx.x, lane = tid & 63, ct = tid >> 6;
  const int nch = K / 32, kspan = K / 2, nst = kspan / kLsKc, k0 = tl.kh * kspan;
  // A: wave-instruction u of wave w reads 4 whole 256-B row segments of the stage (rows 16 w + 4 u +
  // lane / 16, float4 lane % 16): 1 KiB contiguous per row quarter, no partially used lines
  const int a4 = lane & 15;
  int avo[4];
  bool arow[4];
  float asc[4];  // the staged rows' scales 2^s_row
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int rr = 16 * ct + 4 * u + (lane >> 4);
    arow[u] = tl.row0 + rr < B;
    avo[u] = ((tl.row0 + (arow[u] ? rr : 0)) * K + k0 + 4 * a4) * 4;
    asc[u] = bx_pow2(rexp[rr]);
    bad |= a4 == 0 && arow[u] && ls_row_bad(rexp[rr]);
  }
  // B: ls_pack's layout [nb][column tile][chunk][term][lane][8 fp16]: wave-instruction (chunk, term)
  // reads 1 KiB contiguous
  const __amdgpu_buffer_rsrc_t wq = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint16_t *>(wfrag + (size_t)tl.nb * 4 * nch * kLsTerms * 64 * 8), 0, 4 * nch * kLsTerms * 64 * 16,
      0x00020000);
  const int bqo = ((ct * nch * kLsTerms) * 64 + lane) * 16;  // (column tile, chunk 0, term 0, lane), bytes
  constexpr int NVB = 2 * kLsTerms;                          // B loads per stage: (chunk, term)
  lp_f4 va[LZM_LP_DEPTH][4];
  uint4 vb[LZM_LP_DEPTH][NVB];  // global loads LZM_LP_DEPTH - 1 stages ahead
  uint4 wreg[2][kLsTerms];  // the next stage's B fragments (chunk, term) of this wave's column tile
  auto load_stage = [&](int s, lp_f4(&VA)[4], uint4(&VB)[NVB]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 4; ++u)
      VA[u] = arow[u] ? __builtin_bit_cast(lp_f4, __builtin_amdgcn_raw_buffer_load_b128(xr, avo[u], s * kLsKc * 4, 16))
                      : lp_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < NVB; ++u) {  // chunk u / kLsTerms of the stage, term u % kLsTerms
      const int j = (k0 / 32) + 2 * s + u / kLsTerms;
      VB[u] = __builtin_bit_cast(
          uint4, __builtin_amdgcn_raw_buffer_load_b128(wq, bqo, (kLsTerms * j + u % kLsTerms) * 64 * 16, 0));
    }
  };
  auto store_stage = [&](int bsel, const lp_f4(&VA)[4], const uint4(&VB)[NVB]) __attribute__((always_inline)) {
    uint16_t *abuf = lds + bsel * kLsStage;
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // row 16 ct + 4 u + lane / 16: 4 values, half (a4 & 1) of chunk a4 / 2
      const int rr = 16 * ct + 4 * u + (lane >> 4);
      const float v[4] = {VA[u][0], VA[u][1], VA[u][2], VA[u][3]};
      uint32_t hh[2], ll[2];
      ls_split_row<4>(v, asc[u], hh, ll);
      uint16_t *base = abuf + rr * kLsKc + (((a4 >> 1) ^ (rr & 7)) & 7) * 8 + 4 * (a4 & 1);
      *reinterpret_cast<uint2 *>(base) = uint2{hh[0], hh[1]};
      *reinterpret_cast<uint2 *>(base + kLsPlane) = uint2{ll[0], ll[1]};
    }
    // B: a wave loads exactly the fragments its own MFMAs consume, so they stay in registers
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int q = 0; q < kLsTerms; ++q) wreg[c][q] = VB[kLsTerms * c + q];
  };
#pragma unroll
  for (int s0 = 0; s0 < LZM_LP_DEPTH - 1; ++s0)
    if (s0 < nst) load_stage(s0, va[s0], vb[s0]);
  store_stage(0, va[0], vb[0]);
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = bxf4{0.f, 0.f, 0.f, 0.f};
  const int ar = lane & 15, ag = lane >> 4;
  // stage s with register set P = s % LZM_LP_DEPTH (a compile-time index: the loop below is unrolled
  // by the depth); the A planes ping-pong between two LDS buffers (s & 1)
  auto stage = [&](int s, auto par) __attribute__((always_inline)) {
    constexpr int P = decltype(par)::value, D = LZM_LP_DEPTH;
    __syncthreads();
    if (s + D - 1 < nst) load_stage(s + D - 1, va[(P + D - 1) % D], vb[(P + D - 1) % D]);
    const uint16_t *abuf = lds + (s & 1) * kLsStage;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      uint4 a[4][kLsTerms], w[kLsTerms];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int r = 16 * t + ar, o = r * kLsKc + (((4 * c + ag) ^ (r & 7)) & 7) * 8;
#pragma unroll
        for (int tm = 0; tm < kLsTerms; ++tm) a[t][tm] = *reinterpret_cast<const uint4 *>(abuf + tm * kLsPlane + o);
      }
#pragma unroll
      for (int tm = 0; tm < kLsTerms; ++tm) w[tm] = wreg[c][tm];
      // small terms first: l.h, h.l, h.h (ez_lstm_gemm_cell_kernel's order)
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bx_ash(a[t][1]), bx_ash(w[0]), acc[t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bx_ash(a[t][0]), bx_ash(w[1]), acc[t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bx_ash(a[t][0]), bx_ash(w[0]), acc[t], 0, 0, 0);
    }
    // (measured: splitting / storing stage s + 1 BEFORE this stage's MFMAs instead, into the other LDS
    // buffer, made the GEMM slower, 33 K -> 40 K cycles per simulation)
    if (s + 1 < nst) store_stage((s + 1) & 1, va[(P + 1) % D], vb[(P + 1) % D]);
  };
  for (int s = 0; s < nst; s += LZM_LP_DEPTH) {
    stage(s, std::integral_constant<int, 0>());
    if (LZM_LP_DEPTH > 1 && s + 1 < nst) stage(s + 1, std::integral_constant<int, 1 % LZM_LP_DEPTH>());
    if (LZM_LP_DEPTH > 2 && s + 2 < nst) stage(s + 2, std::integral_constant<int, 2 % LZM_LP_DEPTH>());
    if (LZM_LP_DEPTH > 3 && s + 3 < nst) stage(s + 3, std::integral_constant<int, 3 % LZM_LP_DEPTH>());
  }
}

}  // namespace lzm
