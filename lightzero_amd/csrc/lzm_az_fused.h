// lzm_az_fused.h — the whole batched AlphaZero search in ONE launch (fused):
// tree, TicTacToe simulation AND the policy-value network of the TicTacToe config
// (AlphaZeroModel, lzero/model/alphazero_model.py:14-330 with RepresentationNetwork
// common.py:370-460; 16 channels, 3x3 board, value / policy head width 8).
//
// A workgroup of 256 threads (4 waves) owns R boards: their trees live in LDS, the conv weights in
// registers (MFMA B fragments), the head weights in LDS. Per simulation: 16-lane groups descend
// (lzm_az.h's pUCT, tie rule and env replay, on LDS), write the leaf's network input, the 4 waves
// evaluate the R leaves, the groups expand and back up. The roots are evaluated and expanded (with
// the reference's noise) first; the root statistics are finalised (visit_count_to_action_distribution,
// argmax / draw) at the end. One launch per search, no host round trip.
//
// Network (eval mode; BatchNorm folded into the preceding convolution on the host):
//   conv3x3 3->16 +b, ReLU; per residual block: conv3x3 16->16 +b, ReLU, conv3x3 16->16 +b, + x, ReLU
//   (the representation's blocks, then the prediction's); 1x1 conv 16->16 (value) | 16->16 (policy) +b,
//   ReLU; per head: Linear 144->8, LayerNorm(8), ReLU, Linear 8->{1 | 9}; softmax over the 9 logits.
// Convolutions are GEMMs with rows = (board, cell), K = in_channel x tap (im2col gathered from
// zero-bordered 5x5 planes in LDS), N = out channels: v_mfma_f32_16x16x4_f32 (exact f32, a k-ordered
// fmaf chain), K split over the 4 waves, partials summed in wave order. Every output element's
// arithmetic is independent of which tile / workgroup its board lands in, so the standalone
// evaluation kernel (az_net_eval_kernel) and the fused search produce identical bits.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "lzm_az.h"
#include "lzm_tree.h"  // xor_partner, readlane_f

namespace lzm {

constexpr int kAzfThreads = 256;
constexpr int kAzC = 16;      // channels
constexpr int kAzFc = 8;      // head hidden width
constexpr int kAzPlane = 25;  // 5x5 zero-bordered plane
constexpr int kAzBoardX = kAzC * kAzPlane;

typedef float azf4 __attribute__((ext_vector_type(4)));

// head block: value FC1 [8][144], bias, LN gamma, beta, FC2 [8], bias; policy FC1 [8][144], bias, LN
// gamma, beta, FC2 [9][8], bias [9]
constexpr int kAzV1 = 0, kAzV1b = 1152, kAzVg = 1160, kAzVb = 1168, kAzV2 = 1176, kAzV2b = 1184;
constexpr int kAzP1 = 1188, kAzP1b = 2340, kAzPg = 2348, kAzPb = 2356, kAzP2 = 2364, kAzP2b = 2436;
constexpr int kAzHeadFloats = 2448;

// prepared weight buffer (float offsets), see lzm_az_net_prepare
struct AzNetLayout {
  int conv0, conv0_b;      // frag [7][64], bias [16]
  int res, res_b;          // frag [L][36][64], bias [L][16]   (L = 4 * nres conv layers)
  int head, head_b;        // frag [4][2][64], bias [32]
  int heads;               // kAzHeadFloats, inner offsets kAzH* below
  int total;
};

__host__ __device__ inline AzNetLayout az_net_layout(int nres) {
  AzNetLayout L;
  int o = 0;
  auto take = [&](int n) { int r = o; o += (n + 3) & ~3; return r; };
  L.conv0 = take(7 * 64); L.conv0_b = take(16);
  L.res = take(4 * nres * 36 * 64); L.res_b = take(4 * nres * 16);
  L.head = take(4 * 2 * 64); L.head_b = take(32);
  L.heads = take(kAzHeadFloats);
  L.total = o;
  return L;
}

// LDS plan of the network part (floats)
template <int R>
struct AzNetLds {
  static constexpr int T = (9 * R + 15) / 16;            // row tiles
  static constexpr int xin = ((R + 1) * 3 * kAzPlane + 3) & ~3;  // network input planes (+ a zero board), 16-B padded
  static constexpr int xbuf = (R + 1) * kAzBoardX;       // one activation buffer
  static constexpr int hd = R * 32 * 9;                  // 1x1 head outputs [R][32][9]
  static constexpr int red = 4 * T * 2 * 256;            // K-split partials
  static constexpr int heads = kAzHeadFloats;
  static constexpr int out = R * 10;                     // probs [R][9], value [R]
  static constexpr int hid = R * 16;                     // FC1 outputs [R][2][8]
  static constexpr int bias = 16 + 64 * 16 + 32;         // conv biases (<= 16 res layers) + head bias
  static constexpr int total = xin + 3 * xbuf + hd + red + heads + out + hid + bias;
};

template <int R, int NRES>
struct AzNetRegs {
  static constexpr int T = AzNetLds<R>::T;
  float b0[2];                  // conv0 fragments (steps w, w + 4)
  float br[4 * NRES][9];        // 3x3 conv fragments (steps 9w .. 9w + 8)
  float bh[4];                  // 1x1 head fragments (K steps 0..3 of N tile w & 1)
  int koff[9];                  // im2col offsets of this lane's k for steps 9w + j
  int koff0[2];
  int rb[T], rb0[T];            // row base offsets per tile (activation / input planes)
};

struct AzNetSmem {
  float *xin, *x[3], *hd, *red, *heads, *out, *hid, *bias;
};

template <int R>
__device__ inline AzNetSmem az_net_carve(float *p) {
  AzNetSmem s;
  s.xin = p; p += AzNetLds<R>::xin;
  for (int i = 0; i < 3; ++i) { s.x[i] = p; p += AzNetLds<R>::xbuf; }
  s.hd = p; p += AzNetLds<R>::hd;
  s.red = p; p += AzNetLds<R>::red;
  s.heads = p; p += AzNetLds<R>::heads;
  s.out = p; p += AzNetLds<R>::out;
  s.hid = p; p += AzNetLds<R>::hid;
  s.bias = p;
  return s;
}

// zero every plane (borders stay zero forever), stage head weights / biases, load B fragments
template <int R, int NRES>
__device__ inline void az_net_init(const float *__restrict__ w, const AzNetSmem &s, AzNetRegs<R, NRES> &g) {
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  const AzNetLayout L = az_net_layout(NRES);
  const int nzero = AzNetLds<R>::xin + 3 * AzNetLds<R>::xbuf;
  for (int i = tid; i < nzero; i += kAzfThreads) s.xin[i] = 0.0f;
  for (int i = tid; i < kAzHeadFloats; i += kAzfThreads) s.heads[i] = w[L.heads + i];
  for (int i = tid; i < 16; i += kAzfThreads) s.bias[i] = w[L.conv0_b + i];
  for (int i = tid; i < 4 * NRES * 16; i += kAzfThreads) s.bias[16 + i] = w[L.res_b + i];
  for (int i = tid; i < 32; i += kAzfThreads) s.bias[16 + 64 * 16 + i] = w[L.head_b + i];
  const int q = lane >> 4;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int st = wv + 4 * j;
    g.b0[j] = st < 7 ? w[L.conv0 + st * 64 + lane] : 0.0f;
    const int k = 4 * st + q;
    g.koff0[j] = (st < 7 && k < 27) ? (k / 9) * kAzPlane + ((k % 9) / 3) * 5 + (k % 3) : 0;
  }
#pragma unroll
  for (int l = 0; l < 4 * NRES; ++l)
#pragma unroll
    for (int j = 0; j < 9; ++j) g.br[l][j] = w[L.res + (l * 36 + 9 * wv + j) * 64 + lane];
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int k = 4 * (9 * wv + j) + q;
    g.koff[j] = (k / 9) * kAzPlane + ((k % 9) / 3) * 5 + (k % 3);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) g.bh[k] = w[L.head + (k * 2 + (wv & 1)) * 64 + lane];
#pragma unroll
  for (int t = 0; t < AzNetLds<R>::T; ++t) {
    const int m = 16 * t + (lane & 15);
    const int r = m < 9 * R ? m / 9 : R, p = m < 9 * R ? m % 9 : 0;
    g.rb[t] = r * kAzBoardX + (p / 3) * 5 + (p % 3);
    g.rb0[t] = r * 3 * kAzPlane + (p / 3) * 5 + (p % 3);
  }
}

__device__ inline int az_interior(int p) { return (p / 3 + 1) * 5 + (p % 3) + 1; }

// sum the 4 waves' partials in wave order, + bias (+ residual), ReLU, into the interior of `dst`
template <int R>
__device__ inline void az_conv_epilogue(const AzNetSmem &s, const float *bias, const float *res, float *dst) {
  constexpr int T = AzNetLds<R>::T;
  for (int e = threadIdx.x; e < T * 256; e += kAzfThreads) {
    const int t = e >> 8, lane = (e >> 2) & 63, v = e & 3;
    const int m = 16 * t + 4 * (lane >> 4) + v, n = lane & 15;
    if (m >= 9 * R) continue;
    float acc = s.red[(0 * T + t) * 2 * 256 + (e & 255)];
    acc += s.red[(1 * T + t) * 2 * 256 + (e & 255)];
    acc += s.red[(2 * T + t) * 2 * 256 + (e & 255)];
    acc += s.red[(3 * T + t) * 2 * 256 + (e & 255)];
    acc += bias[n];
    const int r = m / 9, p = m % 9;
    const int o = r * kAzBoardX + n * kAzPlane + az_interior(p);
    if (res) acc += res[o];
    dst[o] = acc > 0.0f ? acc : 0.0f;
  }
}

// diagnostics (STAMPS instantiations): thread 0 adds the shader-clock cycles since its last stamp to st[n]
template <bool STAMPS>
__device__ inline void az_stamp(unsigned long long *st, unsigned long long &prev, int n) {
  if (STAMPS && threadIdx.x == 0) {
    const unsigned long long now = __builtin_amdgcn_s_memtime();
    st[n] += now - prev;
    prev = now;
  }
}

// evaluates the R boards whose input planes are in s.xin; leaves probs [R][9] / value [R] in s.out.
// Starts and ends with a workgroup barrier. STAMPS: phases 1 (convolutions), 2 (1x1 heads), 4 (FC1,
// LayerNorm, FC2, softmax) into st[] (thread 0's registers)
template <int R, int NRES, bool STAMPS = false>
__device__ inline void az_net_forward(const AzNetSmem &s, const AzNetRegs<R, NRES> &g,
                                      unsigned long long *st = nullptr, unsigned long long *prev = nullptr) {
  constexpr int T = AzNetLds<R>::T;
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
  unsigned long long pdummy = 0;
  unsigned long long &pv = prev ? *prev : pdummy;
  __syncthreads();
  // ---- conv0: 3 -> 16
  {
    azf4 acc[T];
#pragma unroll
    for (int t = 0; t < T; ++t) {
      acc[t] = azf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if (wv + 4 * j < 7) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(s.xin[g.rb0[t] + g.koff0[j]], g.b0[j], acc[t], 0, 0, 0);
      *(azf4 *)&s.red[((wv * T + t) * 2) * 256 + lane * 4] = acc[t];
    }
  }
  __syncthreads();
  az_conv_epilogue<R>(s, s.bias, nullptr, s.x[0]);
  int cur = 0;
#pragma unroll
  for (int l = 0; l < 4 * NRES; ++l) {
    const int src = (l & 1) ? (cur + 1) % 3 : cur;          // second conv of a block reads the first's output
    const int dst = (l & 1) ? (cur + 2) % 3 : (cur + 1) % 3;
    __syncthreads();
    azf4 acc[T];
#pragma unroll
    for (int t = 0; t < T; ++t) acc[t] = azf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < 9; ++j)
#pragma unroll
      for (int t = 0; t < T; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(s.x[src][g.rb[t] + g.koff[j]], g.br[l][j], acc[t], 0, 0, 0);
#pragma unroll
    for (int t = 0; t < T; ++t) *(azf4 *)&s.red[((wv * T + t) * 2) * 256 + lane * 4] = acc[t];
    __syncthreads();
    az_conv_epilogue<R>(s, s.bias + 16 + l * 16, (l & 1) ? s.x[cur] : nullptr, s.x[dst]);
    if (l & 1) cur = dst;
  }
  __syncthreads();
  az_stamp<STAMPS>(st, pv, 1);
  // ---- 1x1 heads: 16 -> 32 (value 0..15 | policy 16..31). (row tile t, N tile nt) pair p = 2 t + nt runs on
  // wave p % 4 (so nt = wave & 1 and t & 1 = wave >> 1) as one chain of 4 MFMAs over K = 16: no partial sums
  {
    const float *x = s.x[cur];
    const int nt = wv & 1;
#pragma unroll
    for (int t = 0; t < T; ++t) {
      if ((t & 1) != (wv >> 1)) continue;  // wave-uniform
      azf4 acc = azf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(x[g.rb[t] + (4 * k + (lane >> 4)) * kAzPlane + 6], g.bh[k], acc, 0, 0, 0);
      const int n = 16 * nt + (lane & 15);
      const float bn = s.bias[16 + 64 * 16 + n];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int m = 16 * t + 4 * (lane >> 4) + v;
        const float y = acc[v] + bn;
        if (m < 9 * R) s.hd[(m / 9) * 288 + n * 9 + (m % 9)] = y > 0.0f ? y : 0.0f;
      }
    }
  }
  __syncthreads();
  az_stamp<STAMPS>(st, pv, 2);
  // ---- per (board, head) pair, on wave pair % 4: FC1 as 8 units x 8 lanes (18 products per lane, an
  // xor-butterfly sum: every lane of an 8-lane group ends with the same bits), the 8 hidden values to
  // wave-uniform registers, then LayerNorm(8), ReLU, FC2 and (policy) the softmax over lanes 0..8
  const float *hw = s.heads;
  for (int pr = wv; pr < 2 * R; pr += 4) {
    const int r = pr >> 1, head = pr & 1;
    const int j = lane >> 3, q = lane & 7;
    const float *wrow = hw + (head ? kAzP1 : kAzV1) + j * 144 + q * 18;
    const float *in = s.hd + r * 288 + head * 144 + q * 18;
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < 18; ++i) acc = fmaf(wrow[i], in[i], acc);
    acc += xor_partner<1>(acc);
    acc += xor_partner<2>(acc);
    acc += xor_partner<4>(acc);
    acc += hw[(head ? kAzP1b : kAzV1b) + j];
    float h[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) h[u] = readlane_f(acc, 8 * u);
    float mean = 0.0f;
#pragma unroll
    for (int u = 0; u < 8; ++u) mean += h[u];
    mean *= 0.125f;
    float var = 0.0f;
#pragma unroll
    for (int u = 0; u < 8; ++u) var = fmaf(h[u] - mean, h[u] - mean, var);
    var *= 0.125f;
    const float rs = 1.0f / sqrtf(var + 1e-5f);
    float y[8];
    const float *gg = hw + (head ? kAzPg : kAzVg), *bb = hw + (head ? kAzPb : kAzVb);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float z = (h[u] - mean) * rs * gg[u] + bb[u];
      y[u] = z > 0.0f ? z : 0.0f;
    }
    if (head == 0) {
      float v = hw[kAzV2b];
#pragma unroll
      for (int u = 0; u < 8; ++u) v = fmaf(hw[kAzV2 + u], y[u], v);
      if (lane == 0) s.out[R * 9 + r] = v;
    } else {
      const int a = lane & 15;
      float z = -__builtin_inff();
      if (a < 9) {
        z = hw[kAzP2b + a];
#pragma unroll
        for (int u = 0; u < 8; ++u) z = fmaf(hw[kAzP2 + a * 8 + u], y[u], z);
      }
      float mx = z;
      mx = fmaxf(mx, xor_partner<1>(mx));
      mx = fmaxf(mx, xor_partner<2>(mx));
      mx = fmaxf(mx, xor_partner<4>(mx));
      mx = fmaxf(mx, xor_partner<8>(mx));
      const float e = a < 9 ? expf(z - mx) : 0.0f;
      float sum = e;
      sum += xor_partner<1>(sum);
      sum += xor_partner<2>(sum);
      sum += xor_partner<4>(sum);
      sum += xor_partner<8>(sum);
      if (lane < 9) s.out[r * 9 + lane] = e / sum;
    }
  }
  __syncthreads();
  az_stamp<STAMPS>(st, pv, 4);
}

// ---- standalone evaluation: state [n][3][3][3] -> probs [n][9], value [n]
template <int R, int NRES>
__global__ void __launch_bounds__(kAzfThreads) az_net_eval_kernel(const float *__restrict__ w,
                                                                  const float *__restrict__ state, int n,
                                                                  float *probs, float *value) {
  extern __shared__ float az_smem[];
  const AzNetSmem s = az_net_carve<R>(az_smem);
  AzNetRegs<R, NRES> g;
  az_net_init<R, NRES>(w, s, g);
  const int b0 = blockIdx.x * R;
  __syncthreads();
  for (int e = threadIdx.x; e < R * 27; e += kAzfThreads) {
    const int r = e / 27, ch = (e % 27) / 9, p = e % 9;
    s.xin[r * 3 * kAzPlane + ch * kAzPlane + az_interior(p)] = b0 + r < n ? state[(size_t)(b0 + r) * 27 + e % 27] : 0.0f;
  }
  az_net_forward<R, NRES>(s, g);
  for (int e = threadIdx.x; e < R * 10; e += kAzfThreads) {
    const int r = e < R * 9 ? e / 9 : e - R * 9;
    if (b0 + r >= n) continue;
    if (e < R * 9) probs[(size_t)(b0 + r) * 9 + e % 9] = s.out[e];
    else value[b0 + r] = s.out[e];
  }
}

// ---- the fused search
struct AzFusedArgs {
  int B, S, cap, with_noise, sample, export_tree;
  double noise_weight, temperature;
  uint32_t seed;
  const int64_t *counter;
  const float *w;
  const int32_t *boards, *start_index;
  int32_t *visits_out;
  double *probs_out;
  int32_t *action_out;
  AzTree t;  // constants (lut_pb, lut_sqrt, noise) and, when export_tree, the destination of the trees
  unsigned long long *stamps;  // STAMPS instantiations: [0] descend, [1] convolutions, [2] 1x1 heads, [3] 0,
                               // [4] FC1 / LayerNorm / FC2 / softmax, [5] expand + backup, [6] kernel total, [7] sims
};

// group argmax of the pUCT scores (16 lanes): the lowest lane among the maxima (the reference's first strict
// maximum in action order). The double score maps to an order-preserving 64-bit key whose maximum a DPP
// butterfly finds (no LDS round trip); the lowest lane holding it comes from a ballot.
__device__ inline int az_group_argmax(double sc, int gbase) {
  sc += 0.0;  // -0.0 -> +0.0: equal scores, equal keys
  const uint64_t u = __builtin_bit_cast(uint64_t, sc);
  const uint64_t k0 = (u >> 63) ? ~u : (u | 0x8000000000000000ull);
  uint64_t k = k0;
  auto step = [&](auto dd) __attribute__((always_inline)) {
    constexpr int D = decltype(dd)::value;
    const uint32_t lo = (uint32_t)xor_partner<D>((int)(uint32_t)k), hi = (uint32_t)xor_partner<D>((int)(uint32_t)(k >> 32));
    const uint64_t o = ((uint64_t)hi << 32) | lo;
    k = o > k ? o : k;
  };
  step(std::integral_constant<int, 1>());
  step(std::integral_constant<int, 2>());
  step(std::integral_constant<int, 4>());
  step(std::integral_constant<int, 8>());
  return __builtin_ctz(az_group_mask(k0 == k, gbase));
}

// The decision at one node for the 16-lane group: the reference's double pUCT of every child (lane l < n: child
// f + l) and the first maximum (az_group_argmax). pvis: the node's visit count; node: its index (lanes >= n read it,
// so every read is unconditional).
__device__ inline int az_node_decision(const int4 *trec, size_t tb, int node, int f, int n, int pvis, const double *lut_pb,
                                       const double *lut_sq, int l, int gbase) {
  const int4 cr = trec[tb + (l < n ? f + l : node)];
  const double lpb = lut_pb[pvis], lsq = lut_sq[pvis];
  const int cv = cr.y;
  const float q = __int_as_float(cr.z) / (float)(cv > 0 ? cv : 1);
  const float val = cv == 0 ? 0.0f : q;
  double pb = lpb;
  pb *= lsq / (double)(cv + 1);
  double sc = pb * (double)__int_as_float(cr.w) + (double)val;
  sc = l < n ? sc : -__builtin_inf();
  return az_group_argmax(sc, gbase);
}

// get_done_winner_cython.pyx on bit masks of the two players' stones (bit i = cell i). The reference scans
// cells in row-major order and from each stone the directions that stay on the board, returning the first
// full line: a line is only found from its first cell, so the winner is the owner of the full line with the
// lowest first cell; no line and no empty cell is a draw.
__device__ inline void az_done_winner_mask(uint32_t m1, uint32_t m2, int &done, int &winner) {
  constexpr uint32_t kLine[8] = {0x007, 0x049, 0x111, 0x092, 0x054, 0x124, 0x038, 0x1C0};
  constexpr int kStart[8] = {0, 0, 0, 1, 2, 2, 3, 6};  // first cell of each line (ascending)
  winner = -1;
  int first = 9;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    if (kStart[i] >= first) continue;
    if ((m1 & kLine[i]) == kLine[i]) { first = kStart[i]; winner = 1; }
    else if ((m2 & kLine[i]) == kLine[i]) { first = kStart[i]; winner = 2; }
  }
  done = winner != -1 || ((m1 | m2) & 0x1ffu) == 0x1ffu;
}

template <int R, int NRES, bool STAMPS = false>
__global__ void __launch_bounds__(kAzfThreads) az_search_fused_kernel(AzFusedArgs a) {
  extern __shared__ float az_smem[];
  const int tid = threadIdx.x;
  unsigned long long st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const unsigned long long st_begin = STAMPS ? __builtin_amdgcn_s_memtime() : 0ull;
  unsigned long long st_prev = st_begin;
  const int cap = a.cap, S = a.S;
  // ---- LDS: doubles first (alignment), then the tree, then the network
  double *lut_pb = (double *)az_smem;
  double *lut_sq = lut_pb + (S + 1);
  double *noise = lut_sq + (S + 1);
  // node records {meta, visit, value_sum (f32 bits), prior (f32 bits)}: one 16-B LDS read per child, one 8-B
  // read {meta, visit} per node; meta = first child (16 bits, 0xffff: leaf) | nch << 16 | act << 20
  const int ndbl = (2 * (S + 1) + 81 + 1) & ~1;  // the double tables, padded to 16 B
  int4 *trec = (int4 *)(lut_pb + ndbl);
  // the network part 16-B aligned, addressed from az_smem (an integer round trip of the pointer would hide
  // its address space and turn every LDS access of the network into a flat one)
  float *netp = az_smem + 2 * ndbl + 4 * R * cap + 32;  // (+ the path words of the decision refresh)
  const AzNetSmem s = az_net_carve<R>(netp);
  AzNetRegs<R, NRES> g;
  az_net_init<R, NRES>(a.w, s, g);
  for (int i = tid; i <= S; i += kAzfThreads) {
    lut_pb[i] = a.t.lut_pb[i];
    lut_sq[i] = a.t.lut_sqrt[i];
  }
  for (int i = tid; i < 81; i += kAzfThreads) noise[i] = a.t.noise[i];
  const int grp = tid >> 4, l = tid & 15, gbase = (tid & 63) & ~15;
  const int b = blockIdx.x * R + grp;
  const bool active = grp < R && b < a.B;  // group-uniform
  // The group's search state lives in registers (uniform over its 16 lanes unless noted): the root board
  // (lane l < 9: cell l), the node count, and between a descent and its expansion the leaf (node, depth,
  // done, winner, player to move, the move that led to it, lane l < 9: cell l of its board; lane m: the
  // node at depth m of the path)
  int root_cell = 0, root_player = 1, nn = 1;
  int lf_node = 0, lf_depth = 0, lf_done = 0, lf_winner = -1, lf_player = 1, lf_act = 15, lf_cell = 0, lf_path = 0;
  __syncthreads();  // xin zeroed by az_net_init before the roots are written
  if (active) {
    root_player = a.start_index[b] == 0 ? 1 : 2;
    root_cell = l < 9 ? a.boards[(size_t)b * 9 + l] : 0;
    lf_cell = root_cell;
    if (l == 0) {
      trec[grp * cap] = make_int4(0xffff | (15 << 20), 0, __float_as_int(0.0f), __float_as_int(1.0f));
    }
    if (l < 9) {
      float *pl = s.xin + grp * 3 * kAzPlane;
      const int p = az_interior(l);
      pl[p] = root_cell == root_player ? 0.5f : 0.0f;
      pl[kAzPlane + p] = root_cell == 3 - root_player ? 0.5f : 0.0f;
      pl[2 * kAzPlane + p] = 0.5f * (float)root_player;
    }
  }
  const size_t tb = (size_t)grp * cap;
  constexpr bool kCached = R == 1;  // one board per workgroup: cached decisions (below)
  int *s_path = reinterpret_cast<int *>(trec + R * cap);  // [16] the backed-up path, [16] its depth
  for (int sim = -1; sim < S; ++sim) {
    az_stamp<STAMPS>(st, st_prev, 5);
    // ---- descend (sim >= 0): _simulate's walk by the maximal pUCT child, replaying the moves on the
    // group's registers. Child j of a node is the j-th empty cell of the node's board in action order (the
    // expansion creates them so), so the chosen move comes from the board's empty mask, not from the tree.
    if (kCached && sim >= 0 && active) {
      // R = 1: every node's decision is cached in its meta (bits 24..27, refreshed below for each node the last
      // backup touched), so the walk is a chain of one LDS read per level; the move is the child's action
      int cell = root_cell, player = root_player, node = 0, d = 0, act = 15;
      lf_path = 0;
      int meta = trec[tb].x;
      for (; d < kAzPath - 1;) {  // a board fills after 9 moves: bounded descent
        const int f = meta & 0xffff;
        if (f == 0xffff) break;
        node = f + ((meta >> 24) & 15);
        meta = trec[tb + node].x;
        act = (meta >> 20) & 15;
        if (l == act) cell = player;
        player = 3 - player;
        ++d;
        if (l == d) lf_path = node;
      }
      int done, winner;
      az_done_winner_mask(az_group_mask(l < 9 && cell == 1, gbase), az_group_mask(l < 9 && cell == 2, gbase), done,
                          winner);
      lf_node = node; lf_depth = d; lf_done = done; lf_winner = winner; lf_player = player; lf_act = act;
      lf_cell = cell;
      if (l < 9) {
        float *pl = s.xin + grp * 3 * kAzPlane;
        const int p = az_interior(l);
        pl[p] = cell == player ? 0.5f : 0.0f;
        pl[kAzPlane + p] = cell == 3 - player ? 0.5f : 0.0f;
        pl[2 * kAzPlane + p] = 0.5f * (float)player;
      }
    } else if (sim >= 0 && active) {
      int cell = root_cell, player = root_player, node = 0, d = 0, act = 15;
      lf_path = 0;
      for (; d < kAzPath - 1;) {  // a board fills after 9 moves: bounded descent
        // {meta, visit} as one 64-bit value: one LDS round trip before the leaf test and the LUT reads (as two
        // fields the compiler read the visit count only after the test)
        const uint64_t mv = *reinterpret_cast<const uint64_t *>(trec + tb + node);
        const int meta = (int)(uint32_t)mv, pvis = (int)(mv >> 32);
        const int f = meta & 0xffff;
        if (f == 0xffff) break;
        const int n = (meta >> 16) & 15;
        // every read of the level issued at once, no branch: lanes >= n read the node itself
        const int bi = az_node_decision(trec, tb, node, f, n, pvis, lut_pb, lut_sq, l, gbase);
        node = f + bi;
        const uint32_t em = az_group_mask(l < 9 && cell == 0, gbase);
        const bool mine = l < 9 && cell == 0 && __popc(em & ((1u << l) - 1u)) == (uint32_t)bi;
        act = __builtin_ctz(az_group_mask(mine, gbase));
        if (mine) cell = player;
        player = 3 - player;
        ++d;
        if (l == d) lf_path = node;
      }
      int done, winner;
      az_done_winner_mask(az_group_mask(l < 9 && cell == 1, gbase), az_group_mask(l < 9 && cell == 2, gbase), done,
                          winner);
      lf_node = node; lf_depth = d; lf_done = done; lf_winner = winner; lf_player = player; lf_act = act;
      lf_cell = cell;
      if (l < 9) {
        float *pl = s.xin + grp * 3 * kAzPlane;
        const int p = az_interior(l);
        pl[p] = cell == player ? 0.5f : 0.0f;
        pl[kAzPlane + p] = cell == 3 - player ? 0.5f : 0.0f;
        pl[2 * kAzPlane + p] = 0.5f * (float)player;
      }
    }
    az_stamp<STAMPS>(st, st_prev, 0);
    az_net_forward<R, NRES, STAMPS>(s, g, st, &st_prev);
    // ---- expand / back up
    if (active) {
      const float pr = l < 9 ? s.out[grp * 9 + l] : 0.0f;
      if (sim < 0) {
        const bool legal = l < 9 && root_cell == 0;
        const uint32_t gm = az_group_mask(legal, gbase);
        const int n = __popc(gm), rank = __popc(gm & ((1u << l) - 1u));
        if (legal) {
          const size_t c = tb + 1 + rank;
          float p = pr;
          if (a.with_noise) p = (float)((double)pr * (1.0 - a.noise_weight) + noise[(n - 1) * 9 + rank] * a.noise_weight);
          trec[c] = make_int4(0xffff | (l << 20), 0, __float_as_int(0.0f), __float_as_int(p));
        }
        if (l == 0) trec[tb].x = (n > 0 ? 1 : 0xffff) | (n << 16) | (15 << 20);
        nn = 1 + n;
      } else {
        double lv;
        if (!lf_done) {
          const bool legal = l < 9 && lf_cell == 0;
          const uint32_t gm = az_group_mask(legal, gbase);
          const int n = __popc(gm), rank = __popc(gm & ((1u << l) - 1u));
          if (legal) {
            const size_t c = tb + nn + rank;
            trec[c] = make_int4(0xffff | (l << 20), 0, __float_as_int(0.0f), __float_as_int(pr));
          }
          if (l == 0) trec[tb + lf_node].x = (n > 0 ? nn : 0xffff) | (n << 16) | (lf_act << 20);
          nn += n;
          lv = (double)s.out[R * 9 + grp];
        } else {
          lv = lf_winner == -1 ? 0.0 : (lf_player == lf_winner ? 1.0 : -1.0);
        }
        // update_recursive(-leaf_value): lane m updates the path node at depth m, sign by its distance to the leaf
        const float v = (float)(-lv);
        if (l <= lf_depth) {
          int4 &nd = trec[tb + lf_path];
          nd.y += 1;
          nd.z = __float_as_int(__int_as_float(nd.z) + (((lf_depth - l) & 1) ? -v : v));
        }
      }
    }
    if (kCached) {
      // refresh the cached decisions of the nodes whose inputs just changed: a node's pUCT scores depend only on
      // its own visit count and its children's records, which change only when it lies on the backed-up path
      // (the root after its expansion; then path[0 .. depth], the expanded leaf included). One 16-lane group per
      // path node over all four waves, between two barriers: the path's argmaxes in parallel instead of one per
      // level of the next walk. (Measured: wave 0 alone, four nodes per pass and no barriers, 526 vs 502 us per
      // search.)
      if (active && l <= lf_depth) s_path[l] = lf_path;
      if (active && l == 0) s_path[16] = lf_depth;
      __syncthreads();
      const int gi = tid >> 4;
      if (blockIdx.x < a.B && gi <= s_path[16]) {  // group-uniform
        const int node = s_path[gi];
        const uint64_t mv = *reinterpret_cast<const uint64_t *>(trec + node);
        const int meta = (int)(uint32_t)mv, pvis = (int)(mv >> 32);
        const int f = meta & 0xffff, n = (meta >> 16) & 15;
        if (f != 0xffff) {
          const int bi = az_node_decision(trec, 0, node, f, n, pvis, lut_pb, lut_sq, l, gbase);
          if (l == 0) trec[node].x = (meta & ~(15 << 24)) | (bi << 24);
        }
      }
      __syncthreads();
    }
  }
  az_stamp<STAMPS>(st, st_prev, 5);
  if (STAMPS && tid == 0 && a.stamps) {
    st[6] = __builtin_amdgcn_s_memtime() - st_begin;
    st[7] = S;
    for (int n = 0; n < 8; ++n) atomicAdd(a.stamps + n, st[n]);
  }
  // ---- finish: root statistics -> visits / probs / action; optional tree export
  if (active && l == 0) {
    int v[9];
    for (int k = 0; k < 9; ++k) v[k] = 0;
    const int meta = trec[tb].x;
    const int f = meta & 0xffff, n = (meta >> 16) & 15;
    for (int j = 0; f != 0xffff && j < n; ++j) v[(trec[tb + f + j].x >> 20) & 15] = trec[tb + f + j].y;
    az_finalize(b, v, a.temperature, a.sample, a.seed, a.counter, a.visits_out, a.probs_out, a.action_out);
  }
  if (a.export_tree && active) {
    const size_t gb = (size_t)b * cap;
    for (int i = l; i < cap; i += kAzGroup) {
      const bool live = i < nn;
      const int4 rc = trec[tb + i];
      const int meta = rc.x;
      a.t.visit[gb + i] = live ? rc.y : 0;
      a.t.vsum[gb + i] = live ? __int_as_float(rc.z) : 0.0f;
      a.t.prior[gb + i] = live ? __int_as_float(rc.w) : 0.0f;
      a.t.first[gb + i] = live && (meta & 0xffff) != 0xffff ? (meta & 0xffff) : -1;
      a.t.nch[gb + i] = live ? (meta >> 16) & 15 : 0;
      const int act = (meta >> 20) & 15;
      a.t.act[gb + i] = live && act != 15 ? act : -1;
    }
    if (l == 0) a.t.nnodes[b] = nn;
  }
}

}  // namespace lzm
